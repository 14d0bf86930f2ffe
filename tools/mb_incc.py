import sys, numpy as np
sys.path.insert(0, 'cmvs-pmvs_amd'); sys.path.insert(0, 'tests')
import pmvs_amd as P
from conftest import small_scene
inp, p = small_scene(8, 1920, 1080, level=1)
g = P.Scene(inp)
cands = P.synth_candidates(p, inp.projections, 100000, seed=3)
q = np.zeros(len(cands), P.EVAL_QUERY_DTYPE)
for f in ("coord", "normal"): q[f] = cands[f]
q["dscale"] = 0.002; q["num_images"] = 6
V = 8
order = [[v for v in np.argsort(np.abs(np.arange(V) - ref), kind='stable') if v != ref][:5] for ref in range(V)]
for i, c in enumerate(cands):
    ref = int(c["images"][0]); q[i]["images"][:6] = [ref] + order[ref]
for _ in range(3):
    f, st = g.incc_eval(q)
    print(st["kernel_ms"], st["tex_valid"] / len(q))
