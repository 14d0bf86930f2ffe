"""Component timings on the GPU: BOBYQA layouts and the wave-cooperative objective."""
import sys, time, json, numpy as np
sys.path.insert(0, 'cmvs-pmvs_amd'); sys.path.insert(0, 'tests')
import pmvs_amd as P
from conftest import small_scene
res = {}
rng = np.random.default_rng(0)
for mode in (0, 1):
    n = 65536 if mode == 0 else 16384
    x0 = np.zeros((n, 3)); x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
    P.selftest_bobyqa(0, x0[:1024], mode=mode)
    out, ms = P.selftest_bobyqa(0, x0, mode=mode)
    ev = out[:, 4].sum()
    res[f"bobyqa_mode{mode}"] = {"problems": n, "ms": ms, "evals": ev, "evals_per_s": ev / ms * 1e3}
inp, p = small_scene(8, 1920, 1080, level=1)
g = P.Scene(inp)
cands = P.synth_candidates(p, inp.projections, 50000, seed=3)
q = np.zeros(len(cands), P.EVAL_QUERY_DTYPE)
for f in ("coord", "normal"): q[f] = cands[f]
q["dscale"] = 0.002; q["num_images"] = 6
V = 8
for i, c in enumerate(cands):
    ref = int(c["images"][0]); others = [v for v in np.argsort(np.abs(np.arange(V) - ref)) if v != ref][:5]
    q[i]["images"][:6] = [ref] + others
g.incc_eval(q[:1000])
f, st = g.incc_eval(q)
res["incc_eval"] = {"queries": len(q), "ms": st["kernel_ms"], "evals_per_s": len(q) / st["kernel_ms"] * 1e3,
                    "tex_valid": st["tex_valid"]}
print(json.dumps(res, indent=1))
