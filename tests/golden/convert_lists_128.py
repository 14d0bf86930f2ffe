"""One-off conversion of the golden fixtures to the round-3 record layout (PMVS_MAX_IMAGES 64 -> 128;
pmvs_patch lists as int16).  Field values are copied unchanged -- the vectors are the same data,
only the record capacity and the patch list integer width changed.  Run once:
    python tests/golden/convert_lists_128.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402

TARGET = {"refine_in": P.CANDIDATE_DTYPE, "refine_out": P.REFINED_DTYPE, "c1_seeds": P.PATCH_DTYPE,
          "ring8_seeds": P.PATCH_DTYPE}


def convert(a, dt):
    if a.dtype == dt:
        return a
    out = np.zeros(a.shape, dt)
    for f in a.dtype.names:
        src = a[f]
        if src.ndim >= 2 and src.shape[1] != out[f].shape[1]:  # a list field: copy the old capacity
            k = min(src.shape[1], out[f].shape[1])
            if f in ("grids", "vgrids") and dt is P.PATCH_DTYPE:
                out[f][:, :k] = P.grid16(src[:, :k])
            else:
                out[f][:, :k] = src[:, :k]
        elif f in ("grids", "vgrids") and dt is P.PATCH_DTYPE:
            out[f] = P.grid16(src)
        else:
            out[f] = src
    return out


for name in ("ring8", "c1", "seeds"):
    path = os.path.join(HERE, name + ".npz")
    d = dict(np.load(path))
    changed = False
    for k, dt in TARGET.items():
        if k in d and d[k].dtype != dt:
            d[k] = convert(d[k], dt)
            changed = True
    if changed:
        np.savez_compressed(path, **d)
        print("converted", path)
