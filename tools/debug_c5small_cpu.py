"""Diagnostic (CPU only, the oracle half of tools/debug_c5small.py): the 1920x1080 C5-shaped two-cluster exchange (tests/test_gpu_c5_exchange.py) on the device
and in the oracle emulation of tests/test_gpu_c4.py (per-cluster expand + filter, the boundary exchange
in numpy), whole expansions, two iterations; prints each cluster's model size, sphere residuals and the
record mismatches between the two.  python tools/debug_c5small.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import pmvs_amd as P  # noqa: E402
import pyoracle as O  # noqa: E402
from test_gpu_c4 import _grid_wh, _threads, boundary, insert, ring_clusters  # noqa: E402

W, H, LEVEL = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 1)))
world, vpc, ov = 2, 66, 2
clusters = ring_clusters(vpc, world, ov)
full, sp = P.synth_scene(vpc * world, W, H, level=LEVEL, supersample=1, nthreads=16)
cands = P.synth_candidates(sp, full.projections, 5000 * world, seed=0x5EED)
inps = [P.SceneInputs(images=[full.images[i] for i in ids], projections=full.projections[ids], num_targets=len(ids),
                      level=LEVEL) for ids in clusters]
seeds = []
for inp, ids in zip(inps, clusters):
    loc = {v: k for k, v in enumerate(ids)}
    keep = [i for i in range(len(cands)) if int(cands["images"][i][0]) in loc and int(cands["images"][i][1]) in loc]
    cs = cands[keep].copy()
    cs["images"][:, 0] = [loc[int(v)] for v in cs["images"][:, 0]]
    cs["images"][:, 1] = [loc[int(v)] for v in cs["images"][:, 1]]
    o = O.OracleScene(inp)
    r, _ = o.refine_batch(cs, nthreads=8)
    o.close()
    seeds.append(P.patches_from_refined(r))
iterations = 2
# the oracle emulation (tests/test_gpu_c4.py::test_c4_bounded_loop_with_exchange_matches_oracle, whole expansions)
G = world
os_ = [O.OracleScene(inp) for inp in inps]
grids = [_grid_wh(inp) for inp in inps]
tsets = [set(c) for c in clusters]
shared = [[any(v in tsets[q] for q in range(G) if q != r) for v in clusters[r]] for r in range(G)]
models = [s.copy() for s in seeds]
ncc = np.float32(inps[0].threshold)
before = np.float32(ncc - np.float32(0.3))
cthr, depth = 4, 1
O.lib().oracle_set_threads(_threads())
for t in range(iterations):
    for r in range(G):
        o = os_[r]
        o.set_thresholds(float(ncc), float(before), depth)
        m, _, st = o.expand_run(models[r], wave=32768, count_threshold=cthr, cap=len(models[r]) + (4 << 20),
                                after_seeds=(t == 0), min_candidates=131072, nthreads=_threads())
        m, keep, _ = o.filter_run(m)
        models[r] = m[keep == 1]
        print(f"oracle iteration {t + 1} cluster {r}: added {st['added']}, kept {len(models[r])}", flush=True)
    if t + 1 < iterations and os.environ.get("NOEX") is None:
        own = [m[m["fix"] != P.FIX_FOREIGN] for m in models]
        bnd = [boundary(P, own[r], len(clusters[r]), shared[r], *grids[r]) for r in range(G)]
        print(f"oracle boundary sent {[len(b) for b in bnd]}", flush=True)
        models = [np.concatenate([own[r]] + [insert(P, os_[r], bnd[q], clusters[q], clusters[r], len(clusters[r]),
                                                    *grids[r]) for q in range(G) if q != r]) for r in range(G)]
    ncc = np.float32(ncc - np.float32(0.05))
    before = np.float32(before - np.float32(0.05))
    cthr, depth = 2, depth + 1
for o in os_:
    o.close()
want = [m[m["fix"] != P.FIX_FOREIGN] for m in models]
for r in range(G):
    ch = bench.model_checks(want[r], inps[r], ["x"])
    print(f"oracle cluster {r}: {len(want[r])} patches, p99 {ch['sphere_residual_p99']:.4f}, mean {ch['sphere_residual_mean']:.5f}", flush=True)
