"""Time the full expand/filter loop (CFindMatch::run after seeds) on the GPU at a given scale.

usage: python tools/loop_probe.py VIEWS WIDTH HEIGHT LEVEL SEEDS [WAVE]
Prints one line per stage (flushed) so a long run shows progress."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402

V, W, H, L, S = (int(a) for a in sys.argv[1:6])
wave = int(sys.argv[6]) if len(sys.argv) > 6 else 4096
t0 = time.time()
inp, p = P.synth_scene(V, W, H, level=L, supersample=2, nthreads=16)
print(f"synth {time.time() - t0:.1f}s", flush=True)
t0 = time.time()
g = P.Scene(inp)
print(f"scene {time.time() - t0:.1f}s", flush=True)
cands = P.synth_candidates(p, inp.projections, S, seed=11)
t0 = time.time()
r, st = g.refine_batch(cands)
seeds = P.patches_from_refined(r)
print(f"seeds {len(seeds)}/{S} refine {time.time() - t0:.2f}s kernel {st['kernel_ms']:.1f}ms", flush=True)
ncc = np.float32(inp.threshold)
before = np.float32(ncc - np.float32(0.3))
cthr, depth = 4, 1
model = seeds
for it in range(3):
    g.set_thresholds(float(ncc), float(before), depth)
    t0 = time.time()
    model, alive, se = g.expand_run(model, wave=wave, count_threshold=cthr,
                                    after_seeds=it == 0)
    te = time.time() - t0
    print(f"iter {it} expand {te:.2f}s {se}", flush=True)
    t0 = time.time()
    model, keep, sf = g.filter_run(model)
    model = model[keep == 1]
    print(f"iter {it} filter {time.time() - t0:.2f}s kernel {sf['kernel_ms']:.1f}ms kept {len(model)} {sf}", flush=True)
    ncc = np.float32(ncc - np.float32(0.05))
    before = np.float32(before - np.float32(0.05))
    cthr, depth = 2, depth + 1
g.close()
