"""Diagnostic: phase breakdown of the refine kernel on the C2 batch (configs[1]: 8 x 1920x1080,
level 1, 100000 seed-path candidates) with the -DBQ_PROFILE build.  Run on the GPU box:
  PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_prof.so python3 tools/refine_phases.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402

inp, p = P.synth_scene(8, 1920, 1080, level=1, supersample=2, nthreads=16)
s = P.Scene(inp)
c = P.synth_candidates(p, inp.projections, 100000, seed=0x5EED)
s.refine_batch(c)
out, st = s.refine_batch(c)
names = ["refill", "opt_step", "publish", "chunk_setup", "gather", "normalize", "dot", "reduce"]
tot = sum(st["prof"])
print(json.dumps({"config": os.environ.get("PMVS_REFINE_CONFIG", "2408"), "refine_ms": round(st["refine_ms"], 2),
                  "accepted": st["accepted"], "evals": st["evals"], "rounds": st["rounds"], "chunks": st["chunks"],
                  "share": {n: round(v / tot, 4) for n, v in zip(names, st["prof"])},
                  "cycles_per_round": round(tot / max(1, st["rounds"]), 1)}))
