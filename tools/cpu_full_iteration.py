"""One-off measurement for the CPU baseline (round-5 advisor): the CPU oracle runs the WHOLE first
expansion of the C3 loop (all its waves, not the first --cpu-waves) and then one complete CFilter::run
pass over its result, on the bench's own 50-view 3840x2160 scene and seed model, with every CPU this
process may use.  Prints one JSON line: the measured iteration-1 expansion rate, the rate the bench's
extrapolation from its first N waves gives on the same run, the full filter pass's time, and the
filter's per-patch cost beside the bench's sampled estimate.
  python tools/cpu_full_iteration.py [sample_waves=12] [filter_every=8]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import pmvs_amd as P  # noqa: E402
import pyoracle as O  # noqa: E402
import bench  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 12
every = int(sys.argv[2]) if len(sys.argv) > 2 else 8
threads = bench.host_cpus()["usable"]
inp, sp = P.synth_scene(50, 3840, 2160, level=0, supersample=2, nthreads=16, seed=0x504D5653)
scene = P.Scene(inp)
cands = P.synth_candidates(sp, inp.projections, 5000, seed=bench.rank_seed(0))
res, _ = scene.refine_batch(cands)
seeds = P.patches_from_refined(res)
scene.close()
o = O.OracleScene(inp)
ncc, before, depth, cthr = bench.iteration_thresholds(inp.threshold, 0)
o.set_thresholds(ncc, before, depth)
kw = dict(wave=32768, count_threshold=cthr, after_seeds=True, min_candidates=131072, nthreads=threads)
out = {"threads": threads, "seed_patches": int(len(seeds))}
_, _, st = o.expand_run(seeds, cap=len(seeds) + 16 * 32768 * nw + 131072 * nw * 6, max_waves=nw, **kw)
out["sampled"] = {"waves": int(st["waves"]), "added": int(st["added"]), "s": round(o.last_wave_s, 2),
                  "rate": round(st["added"] / o.last_wave_s, 1)}
print(json.dumps(out), flush=True)
t0 = time.time()
m, alive, st = o.expand_run(seeds, cap=len(seeds) + (8 << 20), **kw)
out["full"] = {"waves": int(st["waves"]), "added": int(st["added"]), "s": round(o.last_wave_s, 2),
               "rate": round(st["added"] / o.last_wave_s, 1), "wall_s": round(time.time() - t0, 1)}
out["extrapolation_error"] = round(out["sampled"]["rate"] / out["full"]["rate"] - 1.0, 4)
print(json.dumps(out), flush=True)
model = m[np.asarray(alive).astype(bool)]
del m
sub = model[(model["images"][:, 0] % every) == 0]
O.lib().oracle_set_threads(threads)
t0 = time.perf_counter()
o.filter_run(sub)
ts = time.perf_counter() - t0
t0 = time.perf_counter()
_, keep, counts = o.filter_run(model)
tf = time.perf_counter() - t0
out["filter"] = {"patches": int(len(model)), "s": round(tf, 2), "per_patch_us": round(tf / len(model) * 1e6, 3),
                 "removed": [int(c) for c in counts],
                 "sampled": {"every": every, "patches": int(len(sub)), "s": round(ts, 2),
                             "per_patch_us": round(ts / len(sub) * 1e6, 3)}}
out["filter"]["sample_error"] = round(out["filter"]["sampled"]["per_patch_us"] / out["filter"]["per_patch_us"] - 1.0, 4)
print(json.dumps(out), flush=True)
