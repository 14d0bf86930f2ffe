"""Diagnostic: repeat one expansion case many times on the device (fresh scenes and reused scenes,
with refine batches in between to perturb timing) and count results that differ from the first.
  python3 tools/stress_expand.py DEPTH WAVE REPS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pmvs_amd as P  # noqa: E402

depth, wave, reps = (int(v) for v in sys.argv[1:4])
inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
g0 = P.Scene(inp)
cands = P.synth_candidates(p, inp.projections, 300, seed=3)
r, _ = g0.refine_batch(cands)
pa = P.patches_from_refined(r)
g0.close()
ref = None
bad = 0
for k in range(reps):
    g = P.Scene(inp)
    if k % 3 == 1:
        g.refine_batch(P.synth_candidates(p, inp.projections, 2000, seed=k))
    g.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
    for rep in range(2):
        out, al, st = g.expand_run(pa, wave=wave, cap=100000)
        key = (len(out), st["candidates"], st["added"], out[["coord", "normal", "ncc", "num_images"]].tobytes())
        if ref is None:
            ref = key
            print("first", st, flush=True)
        elif key != ref:
            bad += 1
            print(f"run {k}.{rep}: DIFFERENT n={len(out)} stats={st}", flush=True)
    g.close()
print(f"depth {depth} wave {wave}: {bad} of {2 * reps - 1} repeats differ from the first", flush=True)
