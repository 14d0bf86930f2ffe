"""GPU idle between kernels of the C3 loop, from a rocprofv3 kernel trace (run_kernel_trace.csv):
every gap between one kernel's end and the next kernel's start (serial stream), from the loop's first
empty_blocks_kernel on, summed by the (previous kernel -> next kernel) pair, so that the host
synchronisations that leave the GPU idle are named; and the wave pipeline's per-launch durations split
by the wave's refine form.  python3 tools/ktgaps.py <trace dir> > gaps.json"""
import collections
import csv
import glob
import json
import os
import sys


def short(k):
    name = k.split("(")[0].replace("void ", "")
    if "<" in name:
        name = name.split("<")[0]
    return name.split("::")[-1] or k[:60]


f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
i0 = next(i for i, r in enumerate(rows) if "empty_blocks_kernel" in r["Kernel_Name"])
rows = rows[i0:]
gap, cnt = collections.Counter(), collections.Counter()
busy = 0
end = int(rows[0]["Start_Timestamp"])
prev = "start"
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = short(r["Kernel_Name"])
    if s > end:
        gap[(prev, name)] += s - end
        cnt[(prev, name)] += 1
    busy += e - max(s, end) if e > end else 0
    if e > end:
        end = e
    prev = name
span = end - int(rows[0]["Start_Timestamp"])
# per-launch durations of the wave pipeline's kernels, by the refine form of the wave (the refine kernel
# launched last before them): small waves (lane form) against large ones (split form)
dur = collections.defaultdict(list)
form = "?"
for r in rows:
    name = short(r["Kernel_Name"])
    if name.startswith("refine_"):
        form = name
    if name in ("pre_kernel", "post_kernel", "depth_post_kernel", "refine_lane_kernel", "refine_split_kernel", "prepare_kernel",
                "empty_blocks_kernel", "add_patches_kernel"):
        dur[f"{name} [{form}]"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
by_form = {k: {"launches": len(v), "ms": round(sum(v) / 1e3, 2), "mean_us": round(sum(v) / len(v), 1),
               "median_us": round(sorted(v)[len(v) // 2], 1)} for k, v in sorted(dur.items())}
out = {"span_ms": round(span / 1e6, 3), "busy_ms": round(busy / 1e6, 3), "idle_ms": round((span - busy) / 1e6, 3),
       "launches": len(rows), "by_form": by_form,
       "gaps": [[f"{a} -> {b}", round(v / 1e6, 3), cnt[(a, b)]] for (a, b), v in gap.most_common(40)]}
print(json.dumps(out, indent=0))
