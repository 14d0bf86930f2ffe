"""Diagnostic: the ring8 level-1 filter case with per-stage logging."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "tests")]
import pmvs_amd as P
from test_gpu_filter import make_patch_set
inp, p = P.synth_scene(8, 960, 540, level=1, supersample=2, nthreads=16)
g = P.Scene(inp)
pa = make_patch_set(P, g, inp, p, 100000, 5)
g.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
print("patches", len(pa), flush=True)
try:
    out, keep, st = g.filter_run(pa)
    print(st, flush=True)
except P.PmvsError as e:
    print("error", e, flush=True)
