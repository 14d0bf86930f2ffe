"""Diagnostic: phase breakdown of the refine kernel on the C2 batch (configs[1]: 8 x 1920x1080,
level 1, 100000 seed-path candidates; other batch sizes as arguments) with the -DBQ_PROFILE build.
Run on the GPU box:
  PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_prof.so python3 tools/refine_phases.py [n ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402

inp, p = P.synth_scene(8, 1920, 1080, level=1, supersample=2, nthreads=16)
s = P.Scene(inp)
sizes = [int(a) for a in sys.argv[1:]] or [100000]
c = P.synth_candidates(p, inp.projections, max(sizes), seed=0x5EED)
s.refine_batch(c[:1000])
names = ["refill", "opt_step", "publish", "chunk_setup", "gather", "normalize", "dot", "reduce"]
for n in sizes:
    out, st = s.refine_batch(c[:n])
    tot = sum(st["prof"])
    print(json.dumps({"config": os.environ.get("PMVS_REFINE_CONFIG", "1206"), "n": n, "refine_ms": round(st["refine_ms"], 2),
                      "accepted": st["accepted"], "evals": st["evals"], "rounds": st["rounds"], "chunks": st["chunks"],
                      "share": {k: round(v / max(tot, 1), 4) for k, v in zip(names, st["prof"])},
                      "cycles_per_round": round(tot / max(1, st["rounds"]), 1)}), flush=True)
