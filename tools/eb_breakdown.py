"""Summary of tools/eb_breakdown.sh: per variant, empty_blocks_kernel time (ms) of the launches before
the first prepare_kernel (the first wave's chunks, identical input in every variant)."""
import csv
import glob
import os
import sys

out = sys.argv[1]
for v in ("main", "ebsort", "ebbin", "ebwalk"):
    fs = glob.glob(os.path.join(out, v, "**", "*kernel_trace.csv"), recursive=True)
    if not fs:
        continue
    rows = sorted(csv.DictReader(open(fs[0])), key=lambda r: int(r["Start_Timestamp"]))
    t, n = 0, 0
    for r in rows:
        k = r["Kernel_Name"]
        if "prepare_kernel" in k:
            break
        if "empty_blocks_kernel" in k:
            t += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            n += 1
    print(f"{v:8s} first-wave empty_blocks {t / 1e6:8.2f} ms over {n} launches")
