"""One launch per (mode, kind) of the device BOBYQA self-test, for PMC collection."""
import sys, json, numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'cmvs-pmvs_amd'))
import pmvs_amd as P
rng = np.random.default_rng(0)
n = 16384
x0 = np.zeros((n, 3)); x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
for mode in (0, 1, 3):
    for kind in (0, 1):
        out, ms = P.selftest_bobyqa(kind, x0, mode=mode, maxeval=200)
        print(json.dumps({"mode": mode, "kind": kind, "ms": round(ms, 2), "steps": int(out[:, 4].sum())}), flush=True)
