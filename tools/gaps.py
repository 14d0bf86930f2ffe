"""GPU idle gaps from a rocprofv3 kernel trace (run_kernel_trace.csv): total busy / idle time in a
window and the idle time attributed to (previous kernel -> next kernel) pairs, i.e. where the host
(or a copy) held the GPU up.
    python tools/gaps.py gpurun_out/<tag>/kt/run_kernel_trace.csv [first_kernel last_kernel]
(window: from the first launch whose name starts with first_kernel to the end of the last launch
whose name starts with last_kernel)
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("pmvsdev::", "")
    return n[:48]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    lo, hi = ev[0][0], max(e for _, e, _ in ev)
    if len(sys.argv) > 3:
        lo = min(s for s, _, n in ev if n.startswith(sys.argv[2]))
        hi = max(e for _, e, n in ev if n.startswith(sys.argv[3]))
        ev = [x for x in ev if x[0] >= lo and x[1] <= hi]
    busy, gap = 0, defaultdict(lambda: [0, 0])
    end = ev[0][0]
    prev = "start"
    for s, e, n in ev:
        if s > end:
            g = gap[(prev, n)]
            g[0] += s - end
            g[1] += 1
        busy += max(0, e - max(s, end))
        if e > end:
            end = e
            prev = n
    wall = end - ev[0][0]
    print(f"window {wall / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms ({100 * busy / wall:.1f} %)  idle {(wall - busy) / 1e6:.1f} ms")
    for (p, n), (t, c) in sorted(gap.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{t / 1e6:9.1f} ms {c:6d}x  {p} -> {n}")


if __name__ == "__main__":
    main()
