"""Diagnostic: one filter pass with per-stage progress (PMVS_FILTER_DEBUG=1)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import pmvs_amd as P
from test_gpu_filter import make_patch_set
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
g = P.Scene(inp)
pa = make_patch_set(P, g, inp, p, n, 9, outliers=0.02, fixed=0.01)
print("patches", len(pa), flush=True)
g.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
t = time.time()
out, keep, st = g.filter_run(pa)
print("filter", time.time() - t, st, flush=True)
