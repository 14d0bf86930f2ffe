"""Microbenchmark: device BOBYQA throughput by state placement (mode 0 private/scratch,
2/3/4 = LDS-resident with 16/32/64 problems per workgroup)."""
import sys, json, numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'cmvs-pmvs_amd'))
import pmvs_amd as P
rng = np.random.default_rng(0)
n = 131072
x0 = np.zeros((n, 3)); x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
ref = {}
for mode in (0, 2, 3, 4):
    P.selftest_bobyqa(0, x0[:4096], mode=mode)
    for kind in (0, 1):
        out, ms = P.selftest_bobyqa(kind, x0, mode=mode, maxeval=200)
        same = None
        if mode == 0: ref[kind] = out
        else: same = bool(np.array_equal(out, ref[kind]))
        print(json.dumps({"mode": mode, "kind": kind, "ms": round(ms, 2), "steps": int(out[:, 4].sum()),
                          "Msteps_per_s": round(out[:, 4].sum() / ms / 1e3, 1), "same_as_mode0": same}), flush=True)
