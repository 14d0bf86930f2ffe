"""Print name / calls / total ms / average ms rows of a rocprofv3 run_kernel_stats.csv whose
kernel name matches a regex.   python tools/kstats.py <stats.csv> [regex]"""
import csv
import re
import sys

rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Name"])
    if rx and not rx.search(n):
        continue
    print(f"{n[:60]:60s} {r['Calls']:>6s} {float(r['TotalDurationNs']) / 1e6:10.1f} {float(r['AverageNs']) / 1e6:9.3f}")
