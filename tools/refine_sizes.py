"""Diagnostic: refine-kernel time per batch size and layout on the C3 scene (50 views 3840x2160,
level 0), the launch sizes the C3 loop produces.  One process per library:
  PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_bqp.so python3 tools/refine_sizes.py 2448,2432 5000,20000,80000
prints one JSON line per (config, batch size): refine-kernel ms (HIP events), refined patches/s, and a
hash of the results (every layout must give the same records)."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import numpy as np  # noqa: E402
import pmvs_amd as P  # noqa: E402

cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "1206,132042").split(",")]
sizes = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "2000,5000,10000,20000,40000,80000,120000").split(",")]
t0 = time.time()
inp, sp = P.synth_scene(50, 3840, 2160, level=0, supersample=2, nthreads=16, seed=0x504D5653)
cands = P.synth_candidates(sp, inp.projections, max(sizes), seed=0xC3)
print(f"scene {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
lib = os.path.basename(P.LIB_PATH)
for cfg in cfgs:
    os.environ["PMVS_REFINE_CONFIG"] = str(cfg)
    g = P.Scene(inp)
    g.refine_batch(cands[:2000])  # warm-up
    for n in sizes:
        best = None
        for _ in range(2):
            r, st = g.refine_batch(cands[:n])
            best = st["refine_ms"] if best is None else min(best, st["refine_ms"])
        acc = int((r["status"] == P.ACCEPTED).sum())
        print(json.dumps({"lib": lib, "cfg": cfg, "n": n, "refine_ms": round(best, 3), "accepted": acc,
                          "patches_per_s": round(acc / best * 1e3, 1), "evals": st["evals"],
                          "opt_cycles": st["opt_cycles"], "objective_cycles": st["objective_cycles"],
                          "rounds": st["rounds"], "chunks": st["chunks"], "prof": st["prof"],
                          "sha1": hashlib.sha1(r.tobytes()).hexdigest()[:12]}), flush=True)
    g.close()
