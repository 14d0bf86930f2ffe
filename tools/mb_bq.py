import sys, json, numpy as np
sys.path.insert(0, 'cmvs-pmvs_amd')
import pmvs_amd as P
rng = np.random.default_rng(0)
for n in (65536, 262144, 655360):
    x0 = np.zeros((n, 3)); x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
    P.selftest_bobyqa(0, x0[:4096], mode=0)
    for kind in (0, 1):
        out, ms = P.selftest_bobyqa(kind, x0, mode=0, maxeval=200)
        print(json.dumps({"n": n, "kind": kind, "ms": round(ms, 2), "steps": int(out[:, 4].sum()),
                          "Msteps_per_s": round(out[:, 4].sum() / ms / 1e3, 1)}))
