"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY: ctypes access to the CPU oracle
(oracle/liboracle.so, the restatement of the reference hot path) and to oracle/_ref
(the reference's own camera/option/patch TUs).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cmvs-pmvs_amd"))
import pmvs_amd as P  # noqa: E402  (struct layouts of include/pmvs_amd.h)

ORACLE_LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libpmvs_ref.so")

_lib = None
_ref = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        L = C.CDLL(ORACLE_LIB)
        L.oracle_scene_create.restype = C.c_void_p
        L.oracle_scene_create.argtypes = [C.POINTER(P.SceneDesc)]
        L.oracle_scene_destroy.argtypes = [C.c_void_p]
        L.oracle_is_neighbor.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_set_thresholds.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_int]
        L.oracle_get_level.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_camera.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.oracle_project.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_grab_tex.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_get_color.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_expand_dirs.argtypes = [C.c_void_p] * 3 + [C.c_int, C.c_void_p]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_depth.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_paxes.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_incc_eval.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_refine_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(P.Stats)]
        L.oracle_filter_run.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_expand_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64]
        L.oracle_seed_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_seed_images.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_seed_candidates.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                             C.c_void_p, C.c_int]
        L.oracle_seed_geometry.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                           C.c_void_p, C.c_void_p]
        L.oracle_diag.argtypes = [C.c_void_p, C.c_int]
        L.oracle_list_overflow.argtypes = [C.c_int]
        L.oracle_set_grids.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_lls5.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_bobyqa_test.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_int, C.POINTER(C.c_int)]
        L.oracle_set_grids_images.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 4
        L.oracle_set_grids_full.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 4
        L.oracle_update_depth_maps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_is_visible0.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_check_angles.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 3 + [C.c_float, C.c_float, C.c_void_p]
        L.oracle_distances.argtypes = [C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def ref_lib():
    """The reference's own TUs (None when oracle/_ref was not built: reference absent)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_LIB):
            return None
        R = C.CDLL(REF_LIB)
        R.ref_camera.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p]
        R.ref_project.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        R.ref_option.argtypes = [C.c_char_p, C.c_char_p] + [C.c_void_p] * 7 + [C.c_int]
        R.ref_write_patches.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_int]
        R.ref_write_pset.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        R.ref_ortho.argtypes = [C.c_void_p, C.c_void_p]
        R.ref_get_color.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        R.ref_expand_dirs.argtypes = [C.c_void_p] * 3 + [C.c_int, C.c_void_p]
        R.ref_detect_features.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                          C.c_int]
        R.ref_seed_geometry.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_void_p]
        R.ref_camera_depth.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        _ref = R
    return _ref


def ref_detect_features(rgb, mask=None, edge=None, fcsize=16):
    """The reference's own CHarris + CDifferenceOfGaussians (oracle/_ref) on an RGB8 image:
    float32 [n, 4] = (x, y, response, type) in detectFeatures.cpp order; None if _ref is absent."""
    R = ref_lib()
    if R is None:
        return None
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    e = None if edge is None else np.ascontiguousarray(edge, np.uint8)
    cap = 1 << 16
    while True:
        out = np.zeros((cap, 4), np.float32)
        n = R.ref_detect_features(_p(rgb), _p(m), _p(e), w, h, fcsize, _p(out), cap)
        if n <= cap:
            return out[:n]
        cap = n


def is_neighbor(records):
    """oracle_is_neighbor: the restated isNeighbor / isNeighborRadius on (n, 21) float32 records."""
    r = np.ascontiguousarray(records, np.float32)
    out = np.zeros((len(r), 2), np.int32)
    lib().oracle_is_neighbor(r.ctypes.data, len(r), out.ctypes.data)
    return out


def ref_is_neighbor(records):
    """The reference's own CFindMatch::isNeighbor / isNeighborRadius (oracle/_ref/isneighbor, built
    from findMatch.cpp unmodified) on (n, 21) float32 records; None when _ref is absent."""
    import struct
    import subprocess
    exe = os.path.join(HERE, "_ref", "isneighbor")
    if not os.path.exists(exe):
        return None
    r = np.ascontiguousarray(records, np.float32)
    p = subprocess.run([exe], input=struct.pack("i", len(r)) + r.tobytes(), capture_output=True, check=True)
    return np.frombuffer(p.stdout, np.int32).reshape(len(r), 2).copy()


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _lists(lists):
    off = np.zeros(len(lists) + 1, np.int32)
    for i, l in enumerate(lists):
        off[i + 1] = off[i] + len(l)
    flat = np.array([int(x) for l in lists for x in l] or [0], np.int32)
    return off, flat


def ref_organizer(projections, widths, heights, num_targets, level, csize, ops):
    """The reference's own CPatchOrganizerS / CPhotoSetS (oracle/_ref/organizer, built from
    patchOrganizerS.cpp, photoSetS.cpp, camera.cpp and patch.cpp unmodified) on a scene given by its
    level-0 projections (CONTOUR camera files) and per-level image sizes [V, L]; `ops` as in
    OracleScene.organizer_ops.  Returns one result per op, or None when _ref is absent."""
    import struct
    import subprocess
    import tempfile
    exe = os.path.join(HERE, "_ref", "organizer")
    if not os.path.exists(exe):
        return None
    V, L = np.asarray(widths).shape
    out = bytearray(struct.pack("5i", V, num_targets, level, csize, L))
    with tempfile.TemporaryDirectory() as d:
        for v in range(V):
            path = os.path.join(d, "%08d.txt" % v)
            with open(path, "w") as f:
                f.write("CONTOUR\n")
                for row in projections[v]:
                    f.write(" ".join(repr(float(x)) for x in row) + "\n")
            b = path.encode()
            out += struct.pack("i", len(b)) + b
            out += np.asarray(widths[v], np.int32).tobytes() + np.asarray(heights[v], np.int32).tobytes()
        for op in ops:
            kind = op[0]
            if kind in ("grids_images", "grids"):
                coords, lists = op[1], op[2]
                out += struct.pack("ii", 1 if kind == "grids_images" else 2, len(coords))
                for c, l in zip(coords, lists):
                    out += np.asarray(c, np.float32).tobytes() + struct.pack("i", len(l)) + np.asarray(l, np.int32).tobytes()
            elif kind == "depth":
                out += struct.pack("ii", 3, len(op[1])) + np.ascontiguousarray(op[1], np.float32).tobytes()
            elif kind == "vis0":
                out += struct.pack("ii", 4, len(op[1]))
                for c, t in zip(op[1], op[2]):
                    out += np.asarray(c, np.float32).tobytes() + struct.pack("i", int(t))
            elif kind == "angles":
                coords, lists, lo, hi = op[1:]
                out += struct.pack("iiff", 5, len(coords), lo, hi)
                for c, l in zip(coords, lists):
                    out += np.asarray(c, np.float32).tobytes() + struct.pack("i", len(l)) + np.asarray(l, np.int32).tobytes()
            elif kind == "dist":
                out += struct.pack("i", 6)
        r = subprocess.run([exe], input=bytes(out), capture_output=True, check=True).stdout
    gw = [(int(widths[v][level]) + csize - 1) // csize for v in range(V)]
    gh = [(int(heights[v][level]) + csize - 1) // csize for v in range(V)]
    pos, res = 0, []

    def ints(k):
        nonlocal pos
        a = np.frombuffer(r, np.int32, k, pos).copy()
        pos += 4 * k
        return a
    for op in ops:
        kind = op[0]
        if kind in ("grids_images", "grids"):
            recs = []
            for _ in range(len(op[1])):
                m = int(ints(1)[0])
                recs.append(ints(3 * m).reshape(m, 3))
            res.append(recs)
        elif kind == "depth":
            res.append(ints(sum(gw[t] * gh[t] for t in range(num_targets))))
        elif kind == "vis0":
            res.append(ints(3 * len(op[1])).reshape(-1, 3))
        elif kind == "angles":
            res.append(ints(len(op[1])))
        elif kind == "dist":
            res.append(np.frombuffer(r, np.float32, V * V, pos).reshape(V, V).copy())
            pos += 4 * V * V
    assert pos == len(r), (pos, len(r))
    return res


def _check_lists():
    """The oracle never truncates a list: a result list longer than PMVS_MAX_IMAGES is an error."""
    if lib().oracle_list_overflow(1):
        raise RuntimeError(f"oracle: a patch list exceeded PMVS_MAX_IMAGES ({P.MAX_IMAGES})")


class OracleScene:
    def __init__(self, inputs: "P.SceneInputs"):
        self.inputs = inputs
        self.desc = inputs.build_desc()
        self.h = lib().oracle_scene_create(C.byref(self.desc))
        self.wsize = inputs.wsize

    def close(self):
        if self.h:
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def organizer_ops(self, ops):
        """The restatement's setGridsImages / setGrids / updateDepthMaps / isVisible0 (depth 0) /
        checkAngles / setDistances on the same op list as ref_organizer:
          ("grids_images", coords [n,4], image lists)  -> per record [m, 3] (image, ix, iy)
          ("grids", coords, image lists)                -> the same, every image kept
          ("depth", coords)                             -> every target's cells (patch or -1), concatenated
          ("vis0", coords, images)                      -> [n, 3] (visible, ix, iy)
          ("angles", coords, index lists, min, max)     -> [n] checkAngles
          ("dist",)                                     -> [V, V] setDistances"""
        L = lib()
        res = []
        for op in ops:
            kind = op[0]
            if kind in ("grids_images", "grids"):
                coords = np.ascontiguousarray(op[1], np.float32)
                off, flat = _lists(op[2])
                stride = 3 * P.MAX_IMAGES + 1
                out = np.zeros((len(coords), stride), np.int32)
                fn = L.oracle_set_grids_images if kind == "grids_images" else L.oracle_set_grids_full
                fn(self.h, len(coords), _p(coords), _p(off), _p(flat), _p(out))
                res.append([out[i, 1:1 + 3 * out[i, 0]].reshape(-1, 3) for i in range(len(coords))])
            elif kind == "depth":
                coords = np.ascontiguousarray(op[1], np.float32)
                gw, gh = self.grid_sizes()
                out = np.zeros(int(sum(gw[t] * gh[t] for t in range(self.inputs.num_targets))), np.int32)
                L.oracle_update_depth_maps(self.h, len(coords), _p(coords), _p(out))
                res.append(out)
            elif kind == "vis0":
                coords = np.ascontiguousarray(op[1], np.float32)
                imgs = np.ascontiguousarray(op[2], np.int32)
                out = np.zeros((len(coords), 3), np.int32)
                L.oracle_is_visible0(self.h, len(coords), _p(coords), _p(imgs), _p(out))
                res.append(out)
            elif kind == "angles":
                coords = np.ascontiguousarray(op[1], np.float32)
                off, flat = _lists(op[2])
                out = np.zeros(len(coords), np.int32)
                L.oracle_check_angles(self.h, len(coords), _p(coords), _p(off), _p(flat), op[3], op[4], _p(out))
                res.append(out)
            elif kind == "dist":
                V = len(self.inputs.images)
                out = np.zeros((V, V), np.float32)
                L.oracle_distances(self.h, _p(out))
                res.append(out)
        return res

    def level_sizes(self, levels):
        """Per view, the (width, height) of pyramid levels 0 .. levels-1: [V, L] each."""
        V = len(self.inputs.images)
        w = np.zeros((V, levels), np.int32)
        h = np.zeros((V, levels), np.int32)
        for v in range(V):
            for lv in range(levels):
                a = self.get_level(v, lv)
                h[v, lv], w[v, lv] = a.shape[:2]
        return w, h

    def grid_sizes(self):
        lv, cs = self.inputs.level, self.inputs.csize
        w, h = self.level_sizes(lv + 1)
        return (w[:, lv] + cs - 1) // cs, (h[:, lv] + cs - 1) // cs

    def set_thresholds(self, ncc, before, depth=0):
        lib().oracle_set_thresholds(self.h, ncc, before, depth)

    def get_level(self, view, level):
        w, h = C.c_int(), C.c_int()
        lib().oracle_get_level(self.h, view, level, None, C.byref(w), C.byref(h))
        out = np.empty((h.value, w.value, 3), np.uint8)
        lib().oracle_get_level(self.h, view, level, _p(out), C.byref(w), C.byref(h))
        return out

    def camera(self, view, level):
        out = np.zeros(30, np.float32)
        lib().oracle_camera(self.h, view, level, _p(out))
        return out

    def project(self, view, level, coords):
        coords = np.ascontiguousarray(coords, np.float32)
        out = np.zeros((len(coords), 3), np.float32)
        lib().oracle_project(self.h, view, level, _p(coords), len(coords), _p(out))
        return out

    def get_color(self, view, level, xy):
        xy = np.ascontiguousarray(xy, np.float32)
        out = np.zeros((len(xy), 3), np.float32)
        lib().oracle_get_color(self.h, view, level, _p(xy), len(xy), _p(out))
        return out

    def depth(self, view, coords):
        coords = np.ascontiguousarray(coords, np.float32)
        out = np.zeros(len(coords), np.float32)
        lib().oracle_depth(self.h, view, _p(coords), len(coords), _p(out))
        return out

    def paxes(self, view, coord, normal):
        out = np.zeros(8, np.float32)
        c = np.ascontiguousarray(coord, np.float32)
        n = np.ascontiguousarray(normal, np.float32)
        lib().oracle_paxes(self.h, view, _p(c), _p(n), _p(out))
        return out[:4], out[4:]

    def grab_tex(self, q):
        q = np.ascontiguousarray(q, P.TEX_QUERY_DTYPE)
        out = np.zeros((len(q), 3 * self.wsize * self.wsize), np.float32)
        valid = np.zeros(len(q), np.int32)
        lib().oracle_grab_tex(self.h, _p(q), len(q), _p(out), _p(valid))
        return out, valid

    def incc_eval(self, q, want_encode=False):
        q = np.ascontiguousarray(q, P.EVAL_QUERY_DTYPE)
        out = np.zeros(len(q), np.float64)
        enc = np.zeros((len(q), 3), np.float64) if want_encode else None
        lib().oracle_incc_eval(self.h, _p(q), len(q), _p(out), _p(enc))
        return (out, enc) if want_encode else out

    def filter_run(self, patches):
        """One CFilter::run pass; returns (patches_out, keep, counts[outside, exact, neighbor, groups])."""
        pa = np.ascontiguousarray(patches, P.PATCH_DTYPE).copy()
        keep = np.zeros(len(pa), np.int32)
        counts = np.zeros(4, np.int32)
        lib().oracle_filter_run(self.h, _p(pa), len(pa), _p(keep), _p(counts))
        _check_lists()
        return pa, keep, counts

    def expand_run(self, patches, alive=None, wave=1, count_threshold=4, cap=None, after_seeds=False, min_candidates=0,
                   nthreads=1, max_waves=0):
        """One CExpand::run; returns (patches_out, alive_out, stats dict)."""
        pa = np.ascontiguousarray(patches, P.PATCH_DTYPE)
        al = np.ones(len(pa), np.int32) if alive is None else np.ascontiguousarray(alive, np.int32)
        cap = cap or max(4 * len(pa), 1024)
        out = np.zeros(cap, P.PATCH_DTYPE)
        alo = np.zeros(cap, np.int32)
        st = np.zeros(9, np.int64)
        m = lib().oracle_expand_run(self.h, _p(pa), _p(al), len(pa), wave, count_threshold, int(after_seeds),
                                    int(min_candidates), _p(out), _p(alo), cap,
                                    _p(st), int(nthreads), int(max_waves))
        if m < 0:
            raise RuntimeError("expand_run: capacity too small")
        _check_lists()
        keys = ("parents", "candidates", "fail_prep", "fail_pre", "fail_post", "fail_commit", "added", "waves")
        stats = dict(zip(keys, st.tolist()))
        self.last_wave_s = st[8] / 1e9  # wall time of the waves (not part of the parity dict)
        return out[:m].copy(), alo[:m].copy(), stats

    def run_loop(self, seeds, threshold, iterations=3, wave=4096, cap=None, after_seeds=True, min_candidates=0,
                 nthreads=1, max_waves=0):
        """findMatch.cpp:196-217 after the seed phase, restated: returns (patches, per-iteration counts)."""
        ncc = np.float32(threshold)
        before = np.float32(ncc - np.float32(0.3))  # findMatch.cpp:104
        lib().oracle_set_threads(int(nthreads))
        cthr, depth, model, log = 4, 1, np.ascontiguousarray(seeds, P.PATCH_DTYPE), []
        cap = cap or max(64 * len(model), 1 << 16)
        for t in range(iterations):
            self.set_thresholds(float(ncc), float(before), depth)
            model, _, st_e = self.expand_run(model, wave=wave, count_threshold=cthr, cap=cap,
                                             after_seeds=after_seeds and t == 0, min_candidates=min_candidates,
                                             nthreads=nthreads, max_waves=max_waves)
            model, keep, counts = self.filter_run(model)
            model = model[keep == 1]
            log.append({"depth": depth, "expand": st_e, "filter": counts.tolist(), "patches": len(model)})
            ncc = np.float32(ncc - np.float32(0.05))  # updateThreshold, findMatch.cpp:23-28
            before = np.float32(before - np.float32(0.05))
            cthr, depth = 2, depth + 1
        return model, log

    @staticmethod
    def _points(points):
        """points: list (one per view) of POINT_DTYPE arrays or float32 [n, 4] = (x, y, response, type)."""
        return P.points_flat(points)

    def seed_run(self, points, cap=None):
        """CSeed::run (CPU 1, _response-ordered candidates): (seed patches in addPatch order, stats)."""
        flat, npts = self._points(points)
        cap = cap or max(1024, int(npts.sum()))
        out = np.zeros(cap, P.PATCH_DTYPE)
        st = np.zeros(4, np.int64)
        m = lib().oracle_seed_run(self.h, _p(flat), _p(npts), _p(out), cap, _p(st))
        if m < 0:
            raise RuntimeError("seed_run: capacity too small")
        _check_lists()
        return out[:m].copy(), dict(zip(("trial", "pass", "fail0", "fail1"), st.tolist()))

    def seed_images(self, num_views, num_targets, tau):
        imgs = np.zeros((num_views, tau), np.int32)
        order = np.zeros(num_targets, np.int32)
        lib().oracle_seed_images(self.h, _p(imgs), _p(order))
        return imgs, order

    def seed_candidates(self, points, index, point, cap=1 << 16):
        flat, npts = self._points(points)
        oi = np.zeros((cap, 3), np.int32)
        of = np.zeros((cap, 5), np.float32)
        m = lib().oracle_seed_candidates(self.h, _p(flat), _p(npts), index, point, _p(oi), _p(of), cap)
        if m < 0:
            raise RuntimeError("seed_candidates: capacity too small")
        return oi[:m].copy(), of[:m].copy()

    def seed_geometry(self, i0, i1, xy0, xy1):
        xy0 = np.ascontiguousarray(xy0, np.float32)
        xy1 = np.ascontiguousarray(xy1, np.float32)
        n = len(xy0)
        F = np.zeros(9, np.float64)
        epd = np.zeros(n, np.float32)
        co = np.zeros((n, 4), np.float32)
        lib().oracle_seed_geometry(self.h, i0, i1, _p(xy0), _p(xy1), n, _p(F), _p(epd), _p(co))
        return F.reshape(3, 3), epd, co

    def set_grids(self, patches):
        """CPatchOrganizerS::setGrids on pmvs_patch records (in place)."""
        pa = np.ascontiguousarray(patches, P.PATCH_DTYPE)
        lib().oracle_set_grids(self.h, _p(pa), len(pa))
        return pa

    def refine_batch(self, cands, nthreads=1):
        cands = np.ascontiguousarray(cands, P.CANDIDATE_DTYPE)
        out = np.zeros(len(cands), P.REFINED_DTYPE)
        st = P.Stats()
        lib().oracle_refine_batch(self.h, _p(cands), len(cands), _p(out), nthreads, C.byref(st))
        _check_lists()
        return out, st.as_dict()


def near_threshold(reset=True):
    """Near-threshold decision counts of the oracle since the last reset: constraintImages tests
    (optim.cpp:192-206) within 0.02 of 1 - threshold, filterOutside gains (filter.cpp:62-71) within
    0.05 of 0, refined NCCs within 0.02 of the threshold."""
    out = np.zeros(6, np.int64)
    lib().oracle_diag(_p(out), int(reset))
    return {"constraint_tests": int(out[0]), "constraint_near": int(out[1]), "gains": int(out[2]),
            "gains_near": int(out[3]), "refined": int(out[4]), "ncc_near": int(out[5])}


def lls5(A, b):
    """Cmylapack::lls restated (Eigen JacobiSVD semantics): float32 x[5] for an n x 5 system."""
    A = np.ascontiguousarray(A, np.float32).reshape(-1, 5)
    b = np.ascontiguousarray(b, np.float32)
    x = np.zeros(5, np.float32)
    lib().oracle_lls5(_p(A), _p(b), len(A), _p(x))
    return x


def bobyqa_test(kind, x0, maxeval=1000, maxrec=2000):
    x0 = np.ascontiguousarray(x0, np.float64)
    xo = np.zeros(3)
    fo = np.zeros(1)
    rec = np.zeros(maxrec)
    nrec = C.c_int()
    rc = lib().oracle_bobyqa_test(kind, _p(x0), maxeval, _p(xo), _p(fo), _p(rec), maxrec, C.byref(nrec))
    return rc, xo, fo[0], rec[:min(nrec.value, maxrec)].copy()
