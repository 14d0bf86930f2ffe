#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz -- golden input/output vectors for the PMVS hot path.

Scenes are the deterministic synthetic rings of SURVEY.md §8(d) (pmvs_synth_ring, CPU code
in libpmvs_amd.so; the images themselves are not stored, only their CRC32, since the
renderer regenerates them bit-for-bit).  Expected outputs come from two sources:
  * oracle/_ref (the reference's own camera.cpp compiled unmodified): per-view camera
    centre / optical axis / axes / per-level projection, and CCamera::project of sample
    points -- these vectors are REFERENCE outputs;
  * oracle/liboracle.so (the CPU restatement, pinned on the pieces above): pyramid CRCs,
    grabTex textures, my_f values and full preProcess->refinePatch->postProcess records.
Run from the repo root in the build container:  python tests/golden/make_golden.py
"""
import os
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import pmvs_amd as P  # noqa: E402
import pyoracle as O  # noqa: E402
import pmvs_cases  # noqa: E402

# name: (views, width, height, level, csize, n_tex_cands, n_eval_cands, n_refine)
SCENES = {
    "c1": (3, 640, 480, 2, 4, 60, 60, 300),
    "ring8": (8, 320, 240, 1, 2, 60, 60, 300),
}


def write_contour(path, proj):
    with open(path, "w") as f:
        f.write("CONTOUR\n")
        for row in proj:
            f.write(" ".join(repr(float(v)) for v in row) + "\n")


def ref_cameras(proj, max_level, level_count):
    """Per view: 29 floats per level from the reference CCamera (camera.cpp:13-121)."""
    R = O.ref_lib()
    if R is None:
        raise SystemExit("oracle/_ref not built (reference absent): cannot regenerate reference vectors")
    out = np.zeros((len(proj), level_count, 29), np.float32)
    with tempfile.TemporaryDirectory() as d:
        for v, pm in enumerate(proj):
            path = os.path.join(d, "%08d.txt" % v)
            write_contour(path, pm)
            for lv in range(level_count):
                R.ref_camera(path.encode(), max_level, lv, out[v, lv].ctypes.data)
    return out


def ref_project(proj, max_level, level, pts):
    R = O.ref_lib()
    out = np.zeros((len(proj), len(pts), 3), np.float32)
    with tempfile.TemporaryDirectory() as d:
        for v, pm in enumerate(proj):
            path = os.path.join(d, "%08d.txt" % v)
            write_contour(path, pm)
            R.ref_project(path.encode(), max_level, level, pts.ctypes.data, len(pts), out[v].ctypes.data)
    return out


def make(name, views, width, height, level, csize, ntex, neval, nref):
    inp, p = P.synth_scene(views, width, height, level=level, csize=csize, supersample=2)
    o = O.OracleScene(inp)
    maxlv = level + 3
    g = {"params": np.array([views, width, height, level, csize], np.int64),
         "projections": inp.projections.astype(np.float32),
         "image_crc": np.array([zlib.crc32(im.tobytes()) for im in inp.images], np.uint32)}
    g["pyramid_crc"] = np.array([[zlib.crc32(o.get_level(v, lv).tobytes()) for lv in range(maxlv)]
                                 for v in range(views)], np.uint32)
    g["ref_camera"] = ref_cameras(inp.projections, maxlv, maxlv)
    rng = np.random.default_rng(7)
    pts = np.concatenate([rng.normal(0, 1.0, (200, 3)), np.ones((200, 1))], 1).astype(np.float32)
    pts[150:, 3] = 0.0  # directions (w = 0): the paxes / ray projections
    pts[140:150, :3] *= 50.0  # far and behind-camera points
    g["proj_points"] = pts
    g["ref_project"] = ref_project(inp.projections, maxlv, level, pts)

    tc = P.synth_candidates(p, inp.projections, ntex, seed=101)
    tq = pmvs_cases.tex_queries(o, views, tc)
    tex, valid = o.grab_tex(tq)
    g["tex_query"], g["tex"], g["tex_valid"] = tq, tex, valid

    ec = P.synth_candidates(p, inp.projections, neval, seed=102)
    eq = pmvs_cases.eval_queries(views, ec, per=4, nimg=min(6, views))
    f, enc = o.incc_eval(eq, want_encode=True)
    g["eval_query"], g["eval_f"], g["eval_encode"] = eq, f, enc

    rc = P.synth_candidates(p, inp.projections, nref, seed=103)
    out, st = o.refine_batch(rc, nthreads=8)
    g["refine_in"], g["refine_out"] = rc, out
    g["refine_stats"] = np.array([st[k] for k in ("accepted", "fail_pre", "fail_post", "refine_failed",
                                                  "evals", "tex_valid")], np.int64)
    o.close()
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **g)
    print(f"{path}: {os.path.getsize(path)} B, accepted {st['accepted']}/{nref}, "
          f"valid tex {int(valid.sum())}/{len(tq)}, f<2 {(f < 2).sum()}/{len(eq)}")


if __name__ == "__main__":
    O.build()
    for k, v in SCENES.items():
        make(k, *v)
