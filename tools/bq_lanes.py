"""Optimizer-only cost against chains per wavefront (round 5 design probe).

The BOBYQA self-test kernel runs C problems per 64-lane wavefront, one lane each, state in LDS
(modes: 5 -> C=6, 2 -> 16, 3 -> 32, 6 -> 48, 0 -> 64).  For each C: steps per second over a batch
of many generations (throughput) and over exactly one generation (latency of the slowest wave).
    python tools/bq_lanes.py [kind ...]      (kind 3: timing proxy of the refine objective)
"""
import json
import sys

import numpy as np

sys.path.insert(0, "cmvs-pmvs_amd")
import pmvs_amd as P

MODES = {6: 5, 16: 2, 32: 3, 48: 6, 64: 0}
kinds = [int(k) for k in sys.argv[1:]] or [3, 1]
rng = np.random.default_rng(5)
res = []
for kind in kinds:
    for c, mode in MODES.items():
        for n in (4096, 131072):
            x0 = np.zeros((n, 3))
            x0[:, 0] = rng.uniform(-1, 1, n)
            x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
            P.selftest_bobyqa(kind, x0[:256], mode=mode)
            out, ms = P.selftest_bobyqa(kind, x0, mode=mode)
            ev = out[:, 4]
            waves = (n + c - 1) // c
            wmax = np.array([ev[w * c:(w + 1) * c].max() for w in range(waves)])
            res.append({"kind": kind, "chains_per_wave": c, "n": n, "ms": round(ms, 3),
                        "evals_mean": round(float(ev.mean()), 1), "wave_max_mean": round(float(wmax.mean()), 1),
                        "Msteps_per_s": round(float(ev.sum()) / ms / 1e3, 2),
                        "us_per_wave_step": round(ms * 1e3 / float(wmax.max()), 2) if n == 4096 else None})
            print(json.dumps(res[-1]), flush=True)
