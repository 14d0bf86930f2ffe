"""Diagnostic: run the expansion cases of tests/test_gpu_expand.py with PMVS_POISON_ALLOC set (every
new device allocation filled with a byte pattern) and report, per case, whether the device result
still equals the oracle's (a change means a read of memory no kernel wrote).
  PMVS_POISON_ALLOC=255 python3 tools/flaky_expand.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pmvs_amd as P  # noqa: E402
import pyoracle as O  # noqa: E402
from test_gpu_expand import compare  # noqa: E402

inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
for depth, wave in [(1, 1), (2, 64), (1, 4096), (2, 1), (3, 256)]:
    g = P.Scene(inp)
    o = O.OracleScene(inp)
    cands = P.synth_candidates(p, inp.projections, 300, seed=3)
    r, _ = g.refine_batch(cands)
    pa = P.patches_from_refined(r)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
    out_o, al_o, st_o = o.expand_run(pa, wave=wave, cap=100000)
    out_g, al_g, st_g = g.expand_run(pa, wave=wave, cap=100000)
    try:
        compare(out_g, al_g, st_g, out_o, al_o, st_o)
        res = "OK"
    except AssertionError as e:
        res = f"MISMATCH {e}"
    print(f"poison={os.environ.get('PMVS_POISON_ALLOC')} depth={depth} wave={wave}: {res} gpu={st_g} oracle={st_o}",
          flush=True)
    m, keep, stf = g.filter_run(out_g)
    mo, keepo, cnto = o.filter_run(out_o)
    print(f"   filter: gpu keep {int(keep.sum())} oracle keep {int(keepo.sum())} same={np.array_equal(keep, keepo)}", flush=True)
    g.close()
    o.close()
