"""Per-kernel totals of a rocprofv3 kernel trace (run_kernel_trace.csv) as one JSON object:
{name: [ms, launches]} over the whole trace, plus the first-wave empty_blocks time (the launches
before the first prepare_kernel).  python3 tools/ktsum.py <trace dir> > summary.json"""
import collections
import csv
import glob
import json
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
tot, cnt = collections.Counter(), collections.Counter()
eb_first, seen_prep = 0, False
for r in rows:
    k = r["Kernel_Name"]
    name = k.split("(")[0].replace("void ", "")
    if "<" in name:
        name = name.split("<")[0]
    name = name.split("::")[-1] or k[:60]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[name] += d
    cnt[name] += 1
    if "prepare_kernel" in k:
        seen_prep = True
    if "empty_blocks_kernel" in k and not seen_prep:
        eb_first += d
span = (max(int(r["End_Timestamp"]) for r in rows) - min(int(r["Start_Timestamp"]) for r in rows)) / 1e6
out = {"span_ms": span, "busy_ms": sum(tot.values()) / 1e6, "eb_first_wave_ms": eb_first / 1e6,
       "kernels": {k: [round(v / 1e6, 3), cnt[k]] for k, v in tot.most_common()}}
print(json.dumps(out))
