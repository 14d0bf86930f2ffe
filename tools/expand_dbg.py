"""Diagnose GPU vs oracle expansion differences (prints mismatching patches)."""
import sys, numpy as np
sys.path[:0] = ["cmvs-pmvs_amd", "oracle"]
import pmvs_amd as P, pyoracle as O
depth, wave = int(sys.argv[1]), int(sys.argv[2])
inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
g = P.Scene(inp); o = O.OracleScene(inp)
c = P.synth_candidates(p, inp.projections, 300, seed=3)
r, _ = g.refine_batch(c)
pa = P.patches_from_refined(r)
for sc in (g, o):
    sc.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
og, ag, sg = g.expand_run(pa, wave=wave, cap=100000)
oo, ao, so = o.expand_run(pa, wave=wave, cap=100000)
print("stats g", sg); print("stats o", so)
n = min(len(og), len(oo)); bad = 0
for i in range(n):
    a, b = og[i], oo[i]
    d = [f for f in ("coord", "normal", "ncc", "num_images", "num_vimages", "dflag", "flag")
         if not np.array_equal(np.atleast_1d(a[f]).view(np.uint8), np.atleast_1d(b[f]).view(np.uint8))]
    m = b["num_vimages"]
    if not d and not np.array_equal(a["vimages"][:m], b["vimages"][:m]): d.append("vimages")
    if not d and not np.array_equal(a["vgrids"][:m], b["vgrids"][:m]): d.append("vgrids")
    if d:
        bad += 1
        if bad <= 12:
            print(i, d, "imgs", a["images"][:a["num_images"]], b["images"][:b["num_images"]],
                  "vim", a["vimages"][:a["num_vimages"]], b["vimages"][:m], "vg", a["vgrids"][:a["num_vimages"]].tolist(),
                  b["vgrids"][:m].tolist())
print("mismatching patches", bad, "of", n)
