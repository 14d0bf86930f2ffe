"""Chain lengths of small refine batches (the C3 loop's iterations 2-3 launch ~2.5 k candidates per
wave): per-candidate BOBYQA evaluations, the launch time and the implied latency of one round of the
longest chain, per refine layout.  python tools/small_chains.py [cfg,...] [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import numpy as np  # noqa: E402
import pmvs_amd as P  # noqa: E402

cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "132042,226014").split(",")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2500
inp, sp = P.synth_scene(50, 3840, 2160, level=0, supersample=2, nthreads=16, seed=0x504D5653)
for cfg in cfgs:
    os.environ["PMVS_REFINE_CONFIG"] = str(cfg)
    g = P.Scene(inp)
    for seed in (11, 12, 13):
        cands = P.synth_candidates(sp, inp.projections, n, seed=seed)
        r, st = g.refine_batch(cands)
        ev = r["evals"][r["status"] == P.ACCEPTED]
        print(json.dumps({"cfg": cfg, "seed": seed, "n": n, "refine_ms": round(st["refine_ms"], 3),
                          "evals_max": int(ev.max()), "p99": float(np.percentile(ev, 99)), "p90": float(np.percentile(ev, 90)),
                          "median": float(np.median(ev)), "n_1000": int((ev >= 1000).sum()),
                          "us_per_round_longest": round(st["refine_ms"] * 1e3 / max(1, int(ev.max())), 2)}), flush=True)
    g.close()
