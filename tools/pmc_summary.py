"""Per-kernel sums of a rocprofv3 --pmc run (run_counter_collection.csv): counter totals, dispatch
count and the average per dispatch, as one JSON object (small enough to copy back).
    python tools/pmc_summary.py <dir-with-run_counter_collection.csv> > out.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
out = {k: {"dispatches": len(disp[k]), **{c: v for c, v in sorted(tot[k].items())}} for k in tot}
print(json.dumps(out, indent=1))
