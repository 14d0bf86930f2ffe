#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz -- golden input/output vectors for the PMVS hot path.

Scenes are the deterministic synthetic rings of SURVEY.md §8(d) (pmvs_synth_ring, CPU code
in libpmvs_amd.so; the images themselves are not stored, only their CRC32, since the
renderer regenerates them bit-for-bit).  Expected outputs come from two sources:
  * oracle/_ref (the reference's own camera.cpp compiled unmodified, and its header-inline
    CImage::getColor / isSafe): per-view camera centre / optical axis / axes / per-level
    projection, CCamera::project and computeDepth of sample points, and bilinear getColor
    samples on every pyramid level; the candidate centres of CExpand::findEmptyBlocks
    (expand.cpp:176-177 evaluated with the reference headers, expand_dirs.npz); the Harris and
    DoG feature points of every golden view (harris.cpp / dog.cpp, features.npz); the seed
    phase's setF / computeEPD / triangulation of feature pairs (seeds.npz) -- these vectors are
    REFERENCE outputs;
  * oracle/liboracle.so (the CPU restatement, pinned on the pieces above): pyramid CRCs,
    grabTex textures, my_f values, full preProcess->refinePatch->postProcess records and the
    seed phase's seed patches (seeds.npz).
Run from the repo root in the build container:  python tests/golden/make_golden.py [name ...]
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


def ref_depth(proj, max_level, pts):
    """CCamera::computeDepth (camera.cpp:445-452) per view and point."""
    R = O.ref_lib()
    out = np.zeros((len(proj), len(pts)), np.float32)
    with tempfile.TemporaryDirectory() as d:
        for v, pm in enumerate(proj):
            path = os.path.join(d, "%08d.txt" % v)
            write_contour(path, pm)
            R.ref_camera_depth(path.encode(), max_level, pts.ctypes.data, len(pts), out[v].ctypes.data)
    return out


def color_points(rng, w, h, n):
    """Sample positions inside CImage::isSafe (x in [0, w-2], y in [0, h-2]) incl. the corners,
    integer positions and positions one float ulp below an integer."""
    xy = np.stack([rng.uniform(0, w - 2, n), rng.uniform(0, h - 2, n)], 1).astype(np.float32)
    xy[:8] = np.array([[0, 0], [w - 2, h - 2], [0, h - 2], [w - 2, 0], [1, 1], [w / 2, h / 2],
                       [np.nextafter(np.float32(1), np.float32(0)), 2], [3.5, 2.25]], np.float32)
    xy[8:40] = np.floor(xy[8:40])
    xy[40:72] = np.nextafter(np.ceil(xy[40:72]), np.float32(0))
    return xy


def ref_colors(o, views, maxlv, n=512):
    """CImage::getColor (image.hpp:435-476) of the reference header on the oracle's pyramid levels."""
    R = O.ref_lib()
    rng = np.random.default_rng(11)
    xys, cols = [], []
    for v in range(views):
        for lv in range(maxlv):
            img = np.ascontiguousarray(o.get_level(v, lv))
            h, w = img.shape[:2]
            xy = color_points(rng, w, h, n)
            out = np.zeros((n, 3), np.float32)
            safe = np.zeros(n, np.int32)
            R.ref_get_color(img.ctypes.data, w, h, xy.ctypes.data, n, out.ctypes.data, safe.ctypes.data)
            assert safe.all()
            xys.append(xy)
            cols.append(out)
    return (np.stack(xys).reshape(views, maxlv, n, 2), np.stack(cols).reshape(views, maxlv, n, 3))


def expand_dir_inputs(rng, n=2000):
    """Parent (coord, normal, radius) triples for findEmptyBlocks' candidate centres: random and
    axis-aligned normals (ortho's branches), radii from 1e-3 to 1."""
    coord = np.concatenate([rng.normal(0, 1, (n, 3)), np.ones((n, 1))], 1).astype(np.float32)
    nrm = rng.normal(0, 1, (n, 3))
    nrm[:6] = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    normal = np.concatenate([nrm, np.zeros((n, 1))], 1).astype(np.float32)
    radius = np.exp(rng.uniform(np.log(1e-3), 0, n)).astype(np.float32)
    return coord, normal, radius


def make_expand_dirs():
    R = O.ref_lib()
    coord, normal, radius = expand_dir_inputs(np.random.default_rng(13))
    out = np.zeros((len(coord), 6, 4), np.float32)
    R.ref_expand_dirs(coord.ctypes.data, normal.ctypes.data, radius.ctypes.data, len(coord), out.ctypes.data)
    path = os.path.join(HERE, "expand_dirs.npz")
    np.savez_compressed(path, coord=coord, normal=normal, radius=radius, ref_coords=out)
    print(f"{path}: {os.path.getsize(path)} B")


def isneighbor_records(rng, n):
    """Patch pairs for CFindMatch::isNeighbor / isNeighborRadius (findMatch.cpp:125-185): (n, 21) float32
    records (lhs coord, normal, dscale, rhs coord, normal, dscale, hunit, threshold, radius) with
    random geometry at the scales of a patch model (dscale and hunit ~1e-2 around a unit sphere)."""
    c0 = rng.normal(0, 1, (n, 3))
    n0 = rng.normal(0, 1, (n, 3))
    n0 /= np.linalg.norm(n0, axis=1, keepdims=True)
    tang = rng.normal(0, 1, (n, 3))
    tang -= (tang * n0).sum(1, keepdims=True) * n0
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    ds0 = np.exp(rng.uniform(np.log(2e-3), np.log(2e-2), n))
    ds1 = ds0 * np.exp(rng.uniform(-0.3, 0.3, n))
    hunit = ds0 * np.exp(rng.uniform(-1, 1, n))
    along = rng.uniform(0, 6, n) * hunit
    off = rng.normal(0, 1, n) * ds0 * rng.choice([0.3, 1, 3], n)
    c1 = c0 + along[:, None] * tang + off[:, None] * n0
    ang = rng.uniform(0, np.pi, n) * rng.choice([0.05, 0.3, 1.0], n)
    axis = np.cross(n0, tang)
    n1 = n0 * np.cos(ang)[:, None] + axis * np.sin(ang)[:, None]
    thr = rng.choice([0.5, 1.0, 2.0, 4.0], n)
    radius = hunit * rng.uniform(0.5, 6, n)
    r = np.zeros((n, 21), np.float32)
    r[:, 0:3], r[:, 3] = c0, 1
    r[:, 4:7] = n0
    r[:, 8] = ds0
    r[:, 9:12], r[:, 12] = c1, 1
    r[:, 13:16] = n1
    r[:, 17], r[:, 18], r[:, 19], r[:, 20] = ds1, hunit, thr, radius
    return r


def isneighbor_boundary(rng, n, col, lo, hi, steps=40):
    """Records on the decision boundary of the REFERENCE's isNeighbor (or isNeighborRadius, col 1):
    per record one scalar (the normal offset of rhs, scaled) is bisected between lo and hi until the
    reference's answer flips between adjacent float32 values; both sides are kept."""
    base = isneighbor_records(rng, n)
    d = base[:, 9:12] - base[:, 0:3]
    a = np.full(n, lo, np.float64)
    b = np.full(n, hi, np.float64)

    def at(t):
        r = base.copy()
        r[:, 9:12] = (base[:, 0:3] + d * t[:, None]).astype(np.float32)
        return r
    fa = O.ref_is_neighbor(at(a))[:, col]
    fb = O.ref_is_neighbor(at(b))[:, col]
    keep = fa != fb
    for _ in range(steps):
        m = 0.5 * (a + b)
        fm = O.ref_is_neighbor(at(m))[:, col]
        same = fm == fa
        a = np.where(same, m, a)
        b = np.where(same, b, m)
    return np.concatenate([at(a)[keep], at(b)[keep]])


def make_isneighbor():
    """CFindMatch::isNeighbor / isNeighborRadius of the reference's own findMatch.cpp (compiled
    unmodified in oracle/_ref/isneighbor) on random patch pairs and on pairs bisected onto the
    reference's decision boundaries (threshold, radius, and the 120-degree normal test)."""
    rng = np.random.default_rng(125)
    recs = [isneighbor_records(rng, 3000), isneighbor_boundary(rng, 1000, 0, 0.0, 4.0),
            isneighbor_boundary(rng, 1000, 1, 0.0, 4.0)]
    # normals near 120 degrees apart: lhs . rhs against cos(120 deg) (findMatch.cpp:135)
    r = isneighbor_records(rng, 500)
    r[:, 9:12] = r[:, 0:3]
    n0 = r[:, 4:7].astype(np.float64)
    perp = np.cross(n0, rng.normal(0, 1, (len(r), 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    ang = 2 * np.pi / 3 + rng.normal(0, 1e-6, len(r))
    r[:, 13:16] = (n0 * np.cos(ang)[:, None] + perp * np.sin(ang)[:, None]).astype(np.float32)
    recs.append(r)
    records = np.concatenate(recs).astype(np.float32)
    ref = O.ref_is_neighbor(records)
    path = os.path.join(HERE, "isneighbor.npz")
    np.savez_compressed(path, records=records, ref=ref)
    print(f"{path}: {os.path.getsize(path)} B, {len(records)} pairs, isNeighbor true {int(ref[:, 0].sum())}, "
          f"isNeighborRadius true {int(ref[:, 1].sum())}")


def make_features():
    """CDetectFeatures' two detectors (harris.cpp / dog.cpp compiled unmodified in oracle/_ref) on
    every view of the scene goldens at their option level: REFERENCE outputs (features.npz)."""
    g = {}
    for name, (views, width, height, level, csize, *_rest) in SCENES.items():
        inp, p = P.synth_scene(views, width, height, level=level, csize=csize, supersample=2)
        o = O.OracleScene(inp)
        pts, off = [], [0]
        for v in range(views):
            f = O.ref_detect_features(o.get_level(v, level), fcsize=16)
            pts.append(f)
            off.append(off[-1] + len(f))
        o.close()
        g[f"{name}_points"] = np.concatenate(pts).astype(np.float32)
        g[f"{name}_offsets"] = np.array(off, np.int64)
    path = os.path.join(HERE, "features.npz")
    np.savez_compressed(path, **g)
    print(f"{path}: {os.path.getsize(path)} B, " + ", ".join(f"{k} {len(v)}" for k, v in g.items() if k.endswith("points")))


def ref_seed_geometry(proj, max_level, level, i0, i1, xy0, xy1):
    """Image::setF / computeEPD and the CSeed::unproject triangulation evaluated with the
    reference's CCamera (camera.cpp) and numeric headers (oracle/_ref ref_seed_geometry)."""
    R = O.ref_lib()
    n = len(xy0)
    F = np.zeros(9, np.float64)
    epd = np.zeros(n, np.float32)
    co = np.zeros((n, 4), np.float32)
    with tempfile.TemporaryDirectory() as d:
        p0, p1 = os.path.join(d, "a.txt"), os.path.join(d, "b.txt")
        write_contour(p0, proj[i0])
        write_contour(p1, proj[i1])
        R.ref_seed_geometry(p0.encode(), p1.encode(), max_level, level, xy0.ctypes.data, xy1.ctypes.data, n,
                            F.ctypes.data, epd.ctypes.data, co.ctypes.data)
    return F.reshape(3, 3), epd, co


def make_seeds():
    """Seed phase vectors (seeds.npz): per golden scene, setF / computeEPD / triangulation of feature
    point pairs from the REFERENCE (oracle/_ref), and the oracle's CSeed::run result (seed patches
    in addPatch order + trial/pass/fail counts) on the reference-detected features (regression)."""
    feats = dict(np.load(os.path.join(HERE, "features.npz")))
    g = {}
    rng = np.random.default_rng(17)
    for name, (views, width, height, level, csize, *_rest) in SCENES.items():
        inp, p = P.synth_scene(views, width, height, level=level, csize=csize, supersample=2)
        off = feats[f"{name}_offsets"]
        pts = [feats[f"{name}_points"][off[v]:off[v + 1]] for v in range(views)]
        pairs = [(0, 1), (1, 0), (0, views - 1), (views - 1, 1)]
        F_all, epd_all, co_all, xy_all = [], [], [], []
        for i0, i1 in pairs:
            a = pts[i0][:, :2]
            b = pts[i1][rng.integers(0, len(pts[i1]), len(a)), :2]
            xy0 = np.ascontiguousarray(a, np.float32)
            xy1 = np.ascontiguousarray(b, np.float32)
            F, epd, co = ref_seed_geometry(inp.projections, level + 3, level, i0, i1, xy0, xy1)
            F_all.append(F); epd_all.append(epd); co_all.append(co); xy_all.append(np.stack([xy0, xy1], 1))
        g[f"{name}_pairs"] = np.array(pairs, np.int32)
        g[f"{name}_ref_F"] = np.stack(F_all)
        g[f"{name}_xy"] = np.concatenate(xy_all)
        g[f"{name}_pair_len"] = np.array([len(e) for e in epd_all], np.int64)
        g[f"{name}_ref_epd"] = np.concatenate(epd_all)
        g[f"{name}_ref_coords"] = np.concatenate(co_all)
        o = O.OracleScene(inp)
        seeds, st = o.seed_run(pts)
        o.close()
        g[f"{name}_seeds"] = seeds
        g[f"{name}_seed_stats"] = np.array([st[k] for k in ("trial", "pass", "fail0", "fail1")], np.int64)
        print(f"{name}: {len(seeds)} seeds, {st}")
    path = os.path.join(HERE, "seeds.npz")
    np.savez_compressed(path, **g)
    print(f"{path}: {os.path.getsize(path)} B")


def organizer_cases(o, inp, p, rng, n=600):
    """Inputs of the organizer / photo-set pins: points on and around the synthetic surface
    (candidates jittered along their normals, so several compete for a depth-map cell) and far
    points; image lists of every length; view sets and angle bounds for checkAngles."""
    V = len(inp.images)
    c = P.synth_candidates(p, inp.projections, n, seed=int(rng.integers(1 << 30)))
    coords = c["coord"].astype(np.float32).copy()
    coords[:, :3] += (c["normal"][:, :3] * rng.normal(0, 0.02, (n, 1))).astype(np.float32)
    coords[-40:, :3] = rng.normal(0, 5.0, (40, 3)).astype(np.float32)  # far, often outside every grid
    coords[:, 3] = 1.0
    lists = [sorted(rng.choice(V, int(rng.integers(1, V + 1)), replace=False).tolist()) for _ in range(n)]
    lists = [rng.permutation(l).tolist() for l in lists]
    vis_images = rng.integers(0, inp.num_targets, n).astype(np.int32)
    ang_lists = [rng.choice(V, int(rng.integers(2, min(V, 7) + 1)), replace=False).tolist() for _ in range(n)]
    return coords, lists, vis_images, ang_lists


def organizer_ops(coords, lists, vis_images, ang_lists, min_angle, max_angle):
    return [("grids_images", coords, lists), ("grids", coords, lists), ("depth", coords[:300]),
            ("depth", coords), ("vis0", coords, vis_images), ("angles", coords, ang_lists, min_angle, max_angle),
            ("angles", coords, ang_lists, 0.05, 0.6), ("dist",)]


def make_organizer():
    """CPatchOrganizerS::setGridsImages / setGrids / updateDepthMaps / isVisible0 and
    CPhotoSetS::checkAngles / setDistances of the reference's own patchOrganizerS.cpp /
    photoSetS.cpp (oracle/_ref/organizer) on the ring8 scene."""
    views, width, height, level, csize = SCENES["ring8"][:5]
    inp, p = P.synth_scene(views, width, height, level=level, csize=csize, supersample=2)
    o = O.OracleScene(inp)
    maxlv = level + 3
    w, h = o.level_sizes(maxlv)
    coords, lists, vis_images, ang_lists = organizer_cases(o, inp, p, np.random.default_rng(17))
    min_angle = float(np.float32(inp.max_angle_rad()))
    max_angle = float(np.float32(np.float64(np.float32(60.0)) * np.pi / 180.0))
    ops = organizer_ops(coords, lists, vis_images, ang_lists, min_angle, max_angle)
    ref = O.ref_organizer(inp.projections, w, h, inp.num_targets, level, csize, ops)
    if ref is None:
        raise SystemExit("oracle/_ref/organizer not built (reference absent)")
    o.close()
    off = np.zeros(len(lists) + 1, np.int64)
    off[1:] = np.cumsum([len(l) for l in lists])
    aoff = np.zeros(len(ang_lists) + 1, np.int64)
    aoff[1:] = np.cumsum([len(l) for l in ang_lists])
    g = {"params": np.array([views, width, height, level, csize, inp.num_targets], np.int64),
         "widths": w, "heights": h, "coords": coords, "list_off": off,
         "lists": np.array([x for l in lists for x in l], np.int32), "vis_images": vis_images,
         "ang_off": aoff, "ang_lists": np.array([x for l in ang_lists for x in l], np.int32),
         "angles": np.array([min_angle, max_angle], np.float32)}
    for k, (op, r) in enumerate(zip(ops, ref)):
        if op[0] in ("grids_images", "grids"):
            g[f"ref{k}_n"] = np.array([len(x) for x in r], np.int32)
            g[f"ref{k}"] = np.concatenate(r).astype(np.int32)
        else:
            g[f"ref{k}"] = r
    path = os.path.join(HERE, "organizer.npz")
    np.savez_compressed(path, **g)
    kept = g["ref0_n"].sum()
    print(f"{path}: {os.path.getsize(path)} B, setGridsImages kept {kept} of {off[-1]} entries, "
          f"depth cells set {(g['ref3'] >= 0).sum()}, visible {g['ref4'][:, 0].sum()}/{len(coords)}")


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
    g["ref_depth"] = ref_depth(inp.projections, maxlv, pts)
    g["color_xy"], g["ref_color"] = ref_colors(o, views, maxlv)

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
    if len(sys.argv) > 1:  # named fixtures only, e.g. `make_golden.py organizer`
        for name in sys.argv[1:]:
            globals()["make_" + name]()
        raise SystemExit(0)
    make_organizer()
    make_isneighbor()
    make_expand_dirs()
    make_features()
    make_seeds()
    for k, v in SCENES.items():
        make(k, *v)
