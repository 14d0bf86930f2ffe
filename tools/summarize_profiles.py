#!/usr/bin/env python3
"""Copies the judged rocprofv3 summaries of one gpu_round.sh run from gpurun_out/<tag>/ into
profiles/ and derives the per-launch HBM traffic of the refine kernels.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_bench.json         the bench line of the same call
  profiles/<tag>_pmc.json           FETCH_SIZE / WRITE_SIZE per kernel per launch (bytes)

FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB.  MI355X_MICROARCH.md (HBM section):
on gfx950 FETCH_SIZE counts 64 B per 128-B EA read request, i.e. exactly half the bytes of
wide streaming reads -> multiplied by 2 ("corrected").  Our gathers are 4-B scattered dword
loads, an access width the guide marks uncalibrated; both raw and corrected are recorded.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(dirname, counter):
    out = {}
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            d = out.setdefault(k, {"launches": set(), "kib": 0.0})
            d["launches"].add(r["Dispatch_Id"])
            d["kib"] += float(r["Counter_Value"])
    return {k: {"launches": len(v["launches"]), "bytes_per_launch": v["kib"] * 1024 / max(1, len(v["launches"]))}
            for k, v in out.items()}


def main(tag, workload="c3"):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag.replace('/', '_')}_kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag.replace('/', '_')}_bench.json"))
    fetch = pmc(os.path.join(src, "pmc_fetch"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "pmc_write"), "WRITE_SIZE")
    res = {"source": f"gpurun_out/{tag} (rocprofv3 --pmc, one bench step, {workload} workload)",
           "workload": workload, "fetch_correction": 2.0, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("bytes_per_launch", 0.0)
        w = write.get(k, {}).get("bytes_per_launch", 0.0)
        res["kernels"][k] = {"launches": fetch.get(k, write.get(k, {})).get("launches", 0), "fetch_bytes_raw": f,
                             "fetch_bytes_corrected": 2.0 * f, "write_bytes": w, "hbm_bytes_per_launch": 2.0 * f + w}
    json.dump(res, open(os.path.join(dst, f"{tag.replace('/', '_')}_pmc.json"), "w"), indent=1)
    print(json.dumps(res, indent=1)[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c3")
