"""Deterministic parity cases shared by the CPU golden tests, the GPU parity tests and
tests/golden/make_golden.py: texture-grab and objective-evaluation queries built from
synthetic seed candidates (pmvs_synth_candidates)."""
import numpy as np


def tex_queries(oracle_scene, num_views, cands):
    """Three grabTex queries per candidate: the reference view, the second image and a view
    three steps round the ring (often rejected by the 60-degree / margin tests)."""
    import pmvs_amd as P
    q = np.zeros(len(cands) * 3, P.TEX_QUERY_DTYPE)
    k = 0
    for c in cands:
        ref = int(c["images"][0])
        px, py = oracle_scene.paxes(ref, c["coord"], c["normal"])
        for view in (ref, int(c["images"][1]), (ref + 3) % num_views):
            q[k]["coord"] = c["coord"]
            q[k]["pxaxis"] = px
            q[k]["pyaxis"] = py
            q[k]["normal"] = c["normal"]
            q[k]["view"] = view
            q[k]["normalize"] = k % 2
            k += 1
    return q


def eval_queries(num_views, cands, seed=3, per=4, nimg=6):
    """`per` my_f queries per candidate: x = 0 and random steps in (depth, two angles)."""
    import pmvs_amd as P
    rng = np.random.default_rng(seed)
    q = np.zeros(len(cands) * per, P.EVAL_QUERY_DTYPE)
    nimg = min(nimg, num_views)
    for i, c in enumerate(cands):
        ref = int(c["images"][0])
        others = [int(v) for v in np.argsort(np.abs(np.arange(num_views) - ref), kind="stable") if v != ref]
        for j in range(per):
            r = q[per * i + j]
            r["coord"], r["normal"] = c["coord"], c["normal"]
            r["dscale"] = 0.002 * (1 + j)
            r["num_images"] = nimg
            r["images"][:nimg] = [ref] + others[:nimg - 1]
            r["x"] = rng.normal(0, [2.0, 3.0, 3.0]) if j else [0.0, 0.0, 0.0]
    return q


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 8: np.uint64}[a.dtype.itemsize])
