"""Divergence probe: device BOBYQA lane-mode throughput with identical vs random start points."""
import os, sys, json, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'cmvs-pmvs_amd'))
import pmvs_amd as P
rng = np.random.default_rng(0)
n = 131072
xr = np.zeros((n, 3)); xr[:, 1:] = rng.uniform(-20, 20, (n, 2))
xs = np.tile(xr[:1], (n, 1))
for mode in (0, 2, 4, 1):
    for name, x0 in (("same", xs), ("random", xr)):
        nn = n if mode != 1 else 16384
        P.selftest_bobyqa(0, x0[:4096], mode=mode)
        out, ms = P.selftest_bobyqa(1, x0[:nn], mode=mode, maxeval=200)
        print(json.dumps({"mode": mode, "x0": name, "ms": round(ms, 2), "steps": int(out[:, 4].sum()),
                          "Msteps_per_s": round(out[:, 4].sum() / ms / 1e3, 1)}), flush=True)
