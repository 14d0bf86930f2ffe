"""Host-side view of one C3 step from a rocprofv3 --hip-trace --kernel-trace run (tools/r05q.sh):
the timed pmvs_run_loop (between the last two model_digest_kernel launches: bench.py digests every
step's model), GPU busy/idle in it, and the HIP API calls that took longest inside it, grouped by name.
    python tools/api_gaps.py <dir with run_hip_api_trace.csv and run_kernel_trace.csv>"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
api = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
ker = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
             .replace("pmvsdev::", "")[:40]) for r in ker)
# the timed step: between the last two model digests (bench.py hashes every step's model on the device)
dig = [(s, e) for s, e, n in ev if n.startswith("model_digest_kernel")]
lo, hi = dig[-2][1], dig[-1][0]
w = [x for x in ev if lo <= x[0] <= hi]
busy, e = 0, w[0][0]
for s, t, _ in w:
    busy += max(0, t - max(s, e))
    e = max(e, t)
print(f"window {(hi - lo) / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms, idle {(hi - lo - busy) / 1e6:.1f} ms")
tot = collections.defaultdict(lambda: [0, 0])
big = []
for r in api:
    s, t = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo or s > hi:
        continue
    tot[r["Function"]][0] += 1
    tot[r["Function"]][1] += t - s
    if t - s > 2e6 and r["Function"] != "hipStreamSynchronize":
        big.append(((s - lo) / 1e6, (t - s) / 1e6, r["Function"]))
print("API calls in the window (total ms, calls):")
for k, (n, ns) in sorted(tot.items(), key=lambda x: -x[1][1])[:20]:
    print(f"  {ns / 1e6:9.1f} ms {n:7d}  {k}")
print("non-sync calls over 2 ms:")
for b in big[:60]:
    print(f"  at {b[0]:9.1f} ms  {b[1]:7.2f} ms  {b[2]}")
