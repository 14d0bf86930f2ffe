"""pmvs_amd.py -- host-side Python mirror of the C-ABI in include/pmvs_amd.h (ctypes).

This is the test/bench-facing mirror of the boundary: numpy record dtypes with the exact C
layout of pmvs_candidate / pmvs_refined / pmvs_eval_query / pmvs_tex_query, a Scene wrapper
over pmvs_scene_create/destroy, and the batch entry points.  It never falls back to a CPU
path: if libpmvs_amd.so is missing or a HIP device is absent the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PMVS_AMD_LIB", os.path.join(HERE, "libpmvs_amd.so"))

MAX_IMAGES = 128
MAX_TAU = 16

ACCEPTED, FAIL_PRE, FAIL_POST, FAIL_OVERFLOW = 0, 1, 2, 3
FIX_FOREIGN = 2  # pmvs_patch.fix of another cluster's boundary patch (PMVS_FIX_FOREIGN)

CANDIDATE_DTYPE = np.dtype(
    [("coord", "<f4", 4), ("normal", "<f4", 4), ("dscale", "<f4"), ("num_images", "<i4"),
     ("images", "<i4", MAX_IMAGES)], align=True)
REFINED_DTYPE = np.dtype(
    [("status", "<i4"), ("refine_code", "<i4"), ("evals", "<i4"), ("num_images", "<i4"),
     ("coord", "<f4", 4), ("normal", "<f4", 4), ("ncc", "<f4"), ("dscale", "<f4"), ("ascale", "<f4"),
     ("tmp", "<f4"), ("timages", "<i4"), ("reserved", "<i4"), ("images", "<i4", MAX_IMAGES),
     ("grids", "<i4", (MAX_IMAGES, 2))], align=True)
EVAL_QUERY_DTYPE = np.dtype(
    [("coord", "<f4", 4), ("normal", "<f4", 4), ("dscale", "<f4"), ("num_images", "<i4"),
     ("images", "<i4", MAX_TAU), ("x", "<f8", 3)], align=True)
PATCH_DTYPE = np.dtype(
    [("coord", "<f4", 4), ("normal", "<f4", 4), ("ncc", "<f4"), ("dscale", "<f4"), ("ascale", "<f4"),
     ("tmp", "<f4"), ("timages", "<i4"), ("flag", "<i4"), ("fix", "<i4"), ("num_images", "<i4"),
     ("num_vimages", "<i4"), ("dflag", "<i4"), ("images", "<i2", MAX_IMAGES), ("grids", "<i2", (MAX_IMAGES, 2)),
     ("vimages", "<i2", MAX_IMAGES), ("vgrids", "<i2", (MAX_IMAGES, 2))], align=True)
POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("response", "<f4"), ("type", "<i4")])  # pmvs_point
TEX_QUERY_DTYPE = np.dtype(
    [("coord", "<f4", 4), ("pxaxis", "<f4", 4), ("pyaxis", "<f4", 4), ("normal", "<f4", 4),
     ("view", "<i4"), ("normalize", "<i4")], align=True)


class ViewDesc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.c_void_p), ("mask", C.c_void_p),
                ("edge", C.c_void_p), ("projection", C.c_float * 12)]


class SceneDesc(C.Structure):
    _fields_ = [("num_views", C.c_int32), ("num_targets", C.c_int32), ("level", C.c_int32),
                ("csize", C.c_int32), ("wsize", C.c_int32), ("min_image_num", C.c_int32),
                ("threshold", C.c_float), ("max_angle", C.c_float), ("quad_threshold", C.c_float),
                ("sequence", C.c_int32), ("visdata2_offsets", C.c_void_p), ("visdata2", C.c_void_p),
                ("num_bindexes", C.c_int32), ("bindexes", C.c_void_p), ("views", C.POINTER(ViewDesc))]


class Stats(C.Structure):
    _fields_ = [("candidates", C.c_int64), ("accepted", C.c_int64), ("fail_pre", C.c_int64),
                ("fail_post", C.c_int64), ("refine_failed", C.c_int64), ("evals", C.c_int64),
                ("tex_valid", C.c_int64), ("tex_grabs", C.c_int64), ("kernel_ms", C.c_double),
                ("opt_cycles", C.c_int64), ("objective_cycles", C.c_int64), ("rounds", C.c_int64),
                ("chunks", C.c_int64), ("prof", C.c_int64 * 8), ("pre_ms", C.c_double),
                ("refine_ms", C.c_double), ("post_ms", C.c_double)]

    def as_dict(self):
        return {k: (list(getattr(self, k)) if k == "prof" else getattr(self, k)) for k, _ in self._fields_}


class FilterStats(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("input", "removed_outside", "removed_exact", "removed_neighbor",
                                          "removed_groups", "kept")] + [("kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class ExpandStats(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("parents", "candidates", "fail_prep", "fail_pre", "fail_post",
                                          "fail_commit", "added", "waves")] + [("wall_ms", C.c_double)] + \
               [(k, C.c_int64) for k in ("refined", "evals", "tex_valid")] + [("refine_ms", C.c_double)] + \
               [("refine_launches", C.c_int64), ("tex_valid_small", C.c_int64), ("refine_ms_small", C.c_double),
                ("refine_launches_small", C.c_int64)]

    WORK = ("wall_ms", "refined", "evals", "tex_valid", "refine_ms", "refine_launches", "tex_valid_small",
            "refine_ms_small", "refine_launches_small")  # timing / per-rank work fields

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class LoopIter(C.Structure):
    _fields_ = [("depth", C.c_int32), ("patches", C.c_int32), ("expand", ExpandStats), ("filter", FilterStats),
                ("boundary_sent", C.c_int64), ("boundary_received", C.c_int64), ("boundary_inserted", C.c_int64)]

    def as_dict(self):
        return {"depth": self.depth, "expand": self.expand.as_dict(), "filter": self.filter.as_dict(),
                "patches": self.patches, "boundary": {"sent": self.boundary_sent, "received": self.boundary_received,
                                                      "inserted": self.boundary_inserted}}


class SeedStats(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("trial", "pass_", "fail0", "fail1", "refined", "rounds", "candidates",
                                          "reserved")] + [(k, C.c_double) for k in ("wall_ms", "gen_ms", "refine_ms")]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}
        d["pass"] = d.pop("pass_")
        return d


class Options(C.Structure):
    _fields_ = [(k, C.c_int32) for k in ("level", "csize", "wsize", "min_image_num", "cpu", "use_bound",
                                          "use_vis_data", "sequence", "tflag", "oflag")] + \
               [(k, C.c_float) for k in ("threshold", "set_edge", "max_angle", "quad")] + \
               [(k, C.c_int32) for k in ("num_timages", "num_oimages", "num_bindexes")] + \
               [(k, C.POINTER(C.c_int32)) for k in ("timages", "oimages", "bindexes", "visdata2_offsets",
                                                      "visdata2")]


class SynthParams(C.Structure):
    _fields_ = [("num_views", C.c_int32), ("num_targets", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("supersample", C.c_int32), ("level", C.c_int32),
                ("seed", C.c_uint64), ("ring_radius", C.c_double), ("height_offset", C.c_double),
                ("focal_scale", C.c_double), ("arc_step_deg", C.c_double), ("gain_sigma", C.c_double),
                ("bias_sigma", C.c_double), ("noise_sigma", C.c_double), ("lowtex", C.c_double),
                ("occluder_radius", C.c_double), ("render_first", C.c_int32), ("render_count", C.c_int32)]


# the photometrically hard synthetic mode (pmvs_synth_params): per-view gain / bias, sensor noise,
# low-texture regions and an occluder, so final NCCs spread over ~0.4-1 and image selection
# (constraintImages, optim.cpp:192-206) and filterOutside gains (filter.cpp:62-71) see values near
# their thresholds
HARD = dict(gain_sigma=0.15, bias_sigma=0.04, noise_sigma=0.08, lowtex=0.5, occluder_radius=0.3)


EXPORTS = ["pmvs_last_error", "pmvs_device_count", "pmvs_scene_create", "pmvs_scene_destroy",
           "pmvs_set_thresholds", "pmvs_scene_get_level", "pmvs_grab_tex", "pmvs_incc_eval",
           "pmvs_refine_batch", "pmvs_refine_batch_device", "pmvs_scene_sync", "pmvs_synth_ring",
           "pmvs_synth_candidates", "pmvs_selftest_math", "pmvs_selftest_bobyqa", "pmvs_camera_load",
           "pmvs_ppm_load", "pmvs_options_load", "pmvs_options_free", "pmvs_write_patches", "pmvs_write_pset",
           "pmvs_write_ply", "pmvs_patch_colors", "pmvs_filter_run",
           "pmvs_expand_run", "pmvs_expand_fetch", "pmvs_run_loop", "pmvs_loop_fetch", "pmvs_loop_hash", "pmvs_scene_set_shard", "pmvs_scene_set_shard_rccl", "pmvs_scene_set_cluster",
           "pmvs_scene_set_cluster_rccl", "pmvs_rccl_unique_id",
           "pmvs_rccl_create", "pmvs_rccl_destroy", "pmvs_rccl_allgather", "pmvs_rccl_allgather_device",
           "pmvs_tcp_create", "pmvs_tcp_allgather", "pmvs_tcp_destroy", "pmvs_thread_exchange_create",
           "pmvs_thread_exchange_ctx", "pmvs_thread_allgather", "pmvs_thread_exchange_destroy", "pmvs_detect_features",
           "pmvs_seed_run", "pmvs_seed_fetch", "pmvs_selftest_lls", "pmvs_image_load", "pmvs_pnm_mask_load", "pmvs_set_edge"]

# int fn(void* ctx, const void* send, int64_t bytes, void* recv): all-gather (pmvs_allgather_fn)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)

_lib = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libpmvs_amd.so (raises if it has not been built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run `make -C cmvs-pmvs_amd` (no CPU fallback exists)")
    lib = C.CDLL(path)
    lib.pmvs_last_error.restype = C.c_char_p
    lib.pmvs_device_count.restype = C.c_int32
    lib.pmvs_scene_create.argtypes = [C.POINTER(SceneDesc), C.c_int32, C.POINTER(C.c_void_p)]
    lib.pmvs_scene_destroy.argtypes = [C.c_void_p]
    lib.pmvs_scene_destroy.restype = None
    lib.pmvs_set_thresholds.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_int32]
    lib.pmvs_scene_get_level.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.pmvs_grab_tex.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    lib.pmvs_detect_features.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                         C.POINTER(C.c_int32)]
    lib.pmvs_seed_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                                  C.POINTER(C.c_int32), C.POINTER(SeedStats)]
    lib.pmvs_seed_fetch.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.pmvs_incc_eval.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(Stats)]
    lib.pmvs_refine_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(Stats)]
    lib.pmvs_refine_batch_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.pmvs_scene_sync.argtypes = [C.c_void_p, C.POINTER(Stats)]
    lib.pmvs_synth_ring.argtypes = [C.POINTER(SynthParams), C.c_void_p, C.c_void_p, C.c_int32]
    lib.pmvs_synth_candidates.argtypes = [C.POINTER(SynthParams), C.c_void_p, C.c_int32, C.c_uint64,
                                          C.c_float, C.c_float, C.c_void_p]
    lib.pmvs_selftest_bobyqa.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                         C.c_void_p, C.POINTER(C.c_double)]
    lib.pmvs_selftest_lls.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.pmvs_selftest_math.argtypes = [C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32]
    lib.pmvs_camera_load.argtypes = [C.c_char_p, C.c_void_p]
    lib.pmvs_image_load.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_void_p]
    lib.pmvs_pnm_mask_load.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_void_p]
    lib.pmvs_set_edge.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_float, C.c_void_p]
    lib.pmvs_ppm_load.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_void_p]
    lib.pmvs_options_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.POINTER(Options))]
    lib.pmvs_options_free.argtypes = [C.POINTER(Options)]
    lib.pmvs_options_free.restype = None
    lib.pmvs_write_patches.argtypes = [C.c_char_p, C.c_int32] + [C.c_void_p] * 5
    lib.pmvs_write_pset.argtypes = [C.c_char_p, C.c_int32, C.c_void_p]
    lib.pmvs_write_ply.argtypes = [C.c_char_p, C.c_int32, C.c_void_p, C.c_void_p]
    lib.pmvs_patch_colors.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 4
    lib.pmvs_filter_run.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(FilterStats)]
    lib.pmvs_expand_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(ExpandStats)]
    lib.pmvs_expand_fetch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
    lib.pmvs_run_loop.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_float, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                  C.c_int32, C.POINTER(C.c_int32), C.c_void_p]
    lib.pmvs_loop_fetch.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.pmvs_loop_hash.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    lib.pmvs_scene_set_shard.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    lib.pmvs_scene_set_cluster.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.pmvs_scene_set_cluster_rccl.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    lib.pmvs_rccl_unique_id.argtypes = [C.c_void_p]
    lib.pmvs_rccl_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.pmvs_rccl_destroy.argtypes = [C.c_void_p]
    lib.pmvs_rccl_destroy.restype = None
    lib.pmvs_rccl_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.pmvs_rccl_allgather.restype = C.c_int
    lib.pmvs_scene_set_shard_rccl.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
    lib.pmvs_tcp_create.argtypes = [C.c_int32, C.c_int32, C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    lib.pmvs_tcp_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.pmvs_tcp_destroy.argtypes = [C.c_void_p]
    lib.pmvs_tcp_destroy.restype = None
    lib.pmvs_thread_exchange_create.argtypes = [C.c_int32]
    lib.pmvs_thread_exchange_create.restype = C.c_void_p
    lib.pmvs_thread_exchange_ctx.argtypes = [C.c_void_p, C.c_int32]
    lib.pmvs_thread_exchange_ctx.restype = C.c_void_p
    lib.pmvs_thread_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.pmvs_thread_exchange_destroy.argtypes = [C.c_void_p]
    lib.pmvs_thread_exchange_destroy.restype = None
    for fn in EXPORTS:
        getattr(lib, fn).restype = getattr(lib, fn).restype or C.c_int
    lib.pmvs_last_error.restype = C.c_char_p
    lib.pmvs_device_count.restype = C.c_int32
    lib.pmvs_scene_destroy.restype = None
    lib.pmvs_options_free.restype = None
    lib.pmvs_thread_exchange_create.restype = C.c_void_p
    lib.pmvs_thread_exchange_ctx.restype = C.c_void_p
    lib.pmvs_thread_exchange_destroy.restype = None
    lib.pmvs_tcp_destroy.restype = None
    _lib = lib
    return lib


class PmvsError(RuntimeError):
    pass


def _check(status: int):
    if status != 0:
        msg = load_library().pmvs_last_error().decode(errors="replace")
        raise PmvsError(f"pmvs status {status}: {msg}")


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------------------------- scene
@dataclass
class SceneInputs:
    """Everything pmvs_scene_create needs (SOption + image/camera set), as numpy arrays."""
    images: List[np.ndarray]             # per view uint8 [H, W, 3]
    projections: np.ndarray              # float32 [V, 3, 4] (level 0)
    num_targets: int
    level: int = 1
    csize: int = 2
    wsize: int = 7
    min_image_num: int = 3
    threshold: float = 0.7
    max_angle_deg: Optional[float] = None   # None = SOption default (option.cpp:25)
    quad: float = 2.5
    sequence: int = -1
    visdata2: Optional[List[List[int]]] = None   # None = all-pairs (useVisData 0, option.cpp:204-220)
    bindexes: Sequence[int] = ()
    masks: Optional[List[Optional[np.ndarray]]] = None
    edges: Optional[List[Optional[np.ndarray]]] = None
    _keep: list = field(default_factory=list, repr=False)

    def vis_csr(self):
        V = len(self.images)
        vis = self.visdata2
        if vis is None:
            vis = [[x for x in range(V) if x != y] for y in range(V)]
        off = np.zeros(V + 1, np.int32)
        for i, row in enumerate(vis):
            off[i + 1] = off[i] + len(row)
        flat = np.array([x for row in vis for x in row] or [0], np.int32)
        return off, flat

    def max_angle_rad(self) -> float:
        if self.max_angle_deg is None:
            # SOption(): _maxAngleThreshold = 10.0f * M_PI / 180.0f  (evaluated in double)
            return float(np.float32(np.float64(np.float32(10.0)) * np.pi / np.float64(np.float32(180.0))))
        # SOption::init "maxAngle": _maxAngleThreshold *= M_PI / 180.0f  (float *= double)
        return float(np.float32(np.float64(np.float32(self.max_angle_deg)) * (np.pi / np.float64(np.float32(180.0)))))

    def build_desc(self) -> SceneDesc:
        V = len(self.images)
        self._keep = []
        views = (ViewDesc * V)()
        for i, img in enumerate(self.images):
            img = np.ascontiguousarray(img, dtype=np.uint8)
            assert img.ndim == 3 and img.shape[2] == 3
            self._keep.append(img)
            views[i].width = img.shape[1]
            views[i].height = img.shape[0]
            views[i].rgb = img.ctypes.data
            m = None if self.masks is None else self.masks[i]
            e = None if self.edges is None else self.edges[i]
            if m is not None:
                m = np.ascontiguousarray(m, np.uint8)
                self._keep.append(m)
                views[i].mask = m.ctypes.data
            if e is not None:
                e = np.ascontiguousarray(e, np.uint8)
                self._keep.append(e)
                views[i].edge = e.ctypes.data
            p = np.asarray(self.projections[i], np.float32).reshape(12)
            for k in range(12):
                views[i].projection[k] = float(p[k])
        off, flat = self.vis_csr()
        bidx = np.array(list(self.bindexes) or [0], np.int32)
        self._keep += [off, flat, bidx, views]
        d = SceneDesc()
        d.num_views = V
        d.num_targets = self.num_targets
        d.level = self.level
        d.csize = self.csize
        d.wsize = self.wsize
        d.min_image_num = self.min_image_num
        d.threshold = self.threshold
        d.max_angle = self.max_angle_rad()
        d.quad_threshold = self.quad
        d.sequence = self.sequence
        d.visdata2_offsets = off.ctypes.data
        d.visdata2 = flat.ctypes.data
        d.num_bindexes = len(self.bindexes)
        d.bindexes = bidx.ctypes.data
        d.views = C.cast(views, C.POINTER(ViewDesc))
        return d


class Scene:
    """A device-resident scene on one GPU (pmvs_scene_create)."""

    def __init__(self, inputs: SceneInputs, device: int = 0):
        self.lib = load_library()
        self.inputs = inputs
        self.desc = inputs.build_desc()
        h = C.c_void_p()
        _check(self.lib.pmvs_scene_create(C.byref(self.desc), device, C.byref(h)))
        self.handle = h
        self.wsize = inputs.wsize

    def close(self):
        if getattr(self, "handle", None):
            self.lib.pmvs_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_thresholds(self, ncc: float, ncc_before: float, depth: int = 0):
        _check(self.lib.pmvs_set_thresholds(self.handle, ncc, ncc_before, depth))

    def get_level(self, view: int, level: int) -> np.ndarray:
        w, h = C.c_int32(), C.c_int32()
        _check(self.lib.pmvs_scene_get_level(self.handle, view, level, None, C.byref(w), C.byref(h)))
        out = np.empty((h.value, w.value, 3), np.uint8)
        _check(self.lib.pmvs_scene_get_level(self.handle, view, level, _ptr(out), C.byref(w), C.byref(h)))
        return out

    def detect_features(self, view: int, fcsize: int = 16) -> np.ndarray:
        """CDetectFeatures::run for one view on the device (pmvs_detect_features): POINT_DTYPE
        records, Harris then DoG, each by decreasing response (the reference's order)."""
        n = C.c_int32(0)
        _check(self.lib.pmvs_detect_features(self.handle, view, fcsize, None, 0, C.byref(n)))
        out = np.zeros(n.value, POINT_DTYPE)
        _check(self.lib.pmvs_detect_features(self.handle, view, fcsize, _ptr(out), n.value, C.byref(n)))
        return out

    def seed_run(self, points, batch: int = 0, cap=None):
        """CSeed::run on the device (pmvs_seed_run) from per-view feature points (POINT_DTYPE arrays,
        or float [n, 4] = x, y, response, type): (seed patches in addPatch order, stats)."""
        flat, npts = points_flat(points)
        n = C.c_int32(0)
        st = SeedStats()
        if cap is None:  # the scene keeps the seeds; fetch exactly their number
            _check(self.lib.pmvs_seed_run(self.handle, _ptr(flat), _ptr(npts), int(batch), None, 0, C.byref(n),
                                          C.byref(st)))
            out = np.zeros(n.value, PATCH_DTYPE)
            _check(self.lib.pmvs_seed_fetch(self.handle, _ptr(out), n.value))
            return out, st.as_dict()
        out = np.zeros(int(cap), PATCH_DTYPE)
        _check(self.lib.pmvs_seed_run(self.handle, _ptr(flat), _ptr(npts), int(batch), _ptr(out), int(cap), C.byref(n),
                                      C.byref(st)))
        return out[:n.value].copy(), st.as_dict()

    def grab_tex(self, q: np.ndarray):
        q = np.ascontiguousarray(q, TEX_QUERY_DTYPE)
        n = len(q)
        out = np.zeros((n, 3 * self.wsize * self.wsize), np.float32)
        valid = np.zeros(n, np.int32)
        _check(self.lib.pmvs_grab_tex(self.handle, _ptr(q), n, _ptr(out), _ptr(valid)))
        return out, valid

    def incc_eval(self, q: np.ndarray):
        q = np.ascontiguousarray(q, EVAL_QUERY_DTYPE)
        n = len(q)
        out = np.zeros(n, np.float64)
        st = Stats()
        _check(self.lib.pmvs_incc_eval(self.handle, _ptr(q), n, _ptr(out), C.byref(st)))
        return out, st.as_dict()

    def refine_batch(self, cands: np.ndarray):
        cands = np.ascontiguousarray(cands, CANDIDATE_DTYPE)
        n = len(cands)
        out = np.zeros(n, REFINED_DTYPE)
        st = Stats()
        _check(self.lib.pmvs_refine_batch(self.handle, _ptr(cands), n, _ptr(out), C.byref(st)))
        return out, st.as_dict()

    def refine_batch_device(self, d_in_ptr: int, n: int, d_out_ptr: int):
        _check(self.lib.pmvs_refine_batch_device(self.handle, C.c_void_p(d_in_ptr), n, C.c_void_p(d_out_ptr)))

    def filter_run(self, patches: np.ndarray):
        """One CFilter::run pass on the device: returns (patches_out, keep, stats)."""
        pa = np.ascontiguousarray(patches, PATCH_DTYPE).copy()
        keep = np.zeros(len(pa), np.int32)
        st = FilterStats()
        _check(self.lib.pmvs_filter_run(self.handle, _ptr(pa), len(pa), _ptr(keep), C.byref(st)))
        return pa, keep, st.as_dict()

    def expand_run(self, patches: np.ndarray, alive=None, wave: int = 1, count_threshold: int = 4, cap=None,
                   after_seeds: bool = False, min_candidates: int = 0, max_waves: int = 0):
        """One CExpand::run on the device (expand.cpp:17-406): returns (patches, alive, stats).

        The result holds the input patches (flags updated) followed by the new ones; `cap` bounds
        its size (default: 2^30).  max_waves > 0 stops after that many waves (bounded parity
        samples; PMVS_EXPAND_MAX_WAVES).  Collective when a shard is set (set_shard)."""
        pa = np.ascontiguousarray(patches, PATCH_DTYPE)
        al = np.ones(len(pa), np.int32) if alive is None else np.ascontiguousarray(alive, np.int32)
        cap = int(cap or (1 << 30))
        n_out = C.c_int32(0)
        st = ExpandStats()
        _check(self.lib.pmvs_expand_run(self.handle, _ptr(pa), _ptr(al), len(pa), wave, min_candidates, count_threshold,
                                        int(after_seeds) | (int(max_waves) << 8), None, None, cap, C.byref(n_out),
                                        C.byref(st)))
        out = np.empty(n_out.value, PATCH_DTYPE)
        aout = np.empty(n_out.value, np.int32)
        _check(self.lib.pmvs_expand_fetch(self.handle, _ptr(out), _ptr(aout), n_out.value))
        return out, aout, st.as_dict()

    def set_shard(self, rank: int, world: int, fn=None, ctx=None):
        """Shard the expansion over `world` ranks (pmvs_scene_set_shard); fn is a C function
        pointer (pmvs_allgather_fn: the library's pmvs_thread_allgather, or an ALLGATHER_FN
        callback such as DistExchange's).  The callback object must outlive the scene's use."""
        self._shard_keep = fn
        ptr = None if fn is None else (fn if isinstance(fn, int) else C.cast(fn, C.c_void_p).value)
        _check(self.lib.pmvs_scene_set_shard(self.handle, rank, world, ptr, ctx))

    def set_cluster(self, rank: int, world: int, image_ids, fn=None, ctx=None):
        """One CMVS cluster of `world` (pmvs_scene_set_cluster): run_loop then exchanges boundary
        patches with the other ranks after every iteration.  image_ids: the global image number of
        each view.  fn: a pmvs_allgather_fn (ThreadExchange.endpoint / DistExchange.fn).  Collective."""
        ids = np.ascontiguousarray(image_ids, np.int32)
        assert len(ids) == len(self.inputs.images)
        self._cluster_keep = (fn, ids)
        ptr = None if fn is None else (fn if isinstance(fn, int) else C.cast(fn, C.c_void_p).value)
        _check(self.lib.pmvs_scene_set_cluster(self.handle, rank, world, _ptr(ids), ptr, ctx))

    def run_loop(self, seeds: np.ndarray, threshold: float, iterations: int = 3, wave: int = 4096, cap=None,
                 after_seeds: bool = True, native: bool = True, min_candidates: int = 0, max_waves: int = 0,
                 fetch: bool = True):
        """CFindMatch::run after the seed phase (findMatch.cpp:196-217): depth 1, then `iterations` x
        (CExpand::run, CFilter::run, updateThreshold, ++depth).  Thresholds follow the reference's
        float arithmetic: before = threshold - 0.3f (findMatch.cpp:104), -= 0.05f per iteration and
        _countThreshold1 4 -> 2 (findMatch.cpp:23-28).  native=True runs the whole loop in the
        library with the model resident in HBM (pmvs_run_loop); native=False composes expand_run
        and filter_run through host memory (same result).  max_waves > 0 bounds every iteration's
        expansion to that many waves (PMVS_EXPAND_MAX_WAVES: bounded full-size parity samples).
        Returns (patches, per-iteration stats).  fetch=False (native only) leaves the result on the
        device and returns (its size, stats): loop_hash() / loop_fetch(n) then read it."""
        model = np.ascontiguousarray(seeds, PATCH_DTYPE)
        if native:
            iters = (LoopIter * max(1, iterations))()
            n_out = C.c_int32(0)
            _check(self.lib.pmvs_run_loop(self.handle, _ptr(model), len(model), float(np.float32(threshold)),
                                          iterations, wave, min_candidates,
                                          (1 if after_seeds else 0) | (int(max_waves) << 8), int(cap or (1 << 30)),
                                          C.byref(n_out), iters))
            log = [iters[t].as_dict() for t in range(iterations)]
            if not fetch:
                return n_out.value, log
            return self.loop_fetch(n_out.value), log
        ncc = np.float32(threshold)
        before = np.float32(ncc - np.float32(0.3))
        cthr, depth = 4, 1
        log = []
        for t in range(iterations):
            self.set_thresholds(float(ncc), float(before), depth)
            model, alive, st_e = self.expand_run(model, wave=wave, count_threshold=cthr, cap=cap,
                                                 after_seeds=after_seeds and t == 0, min_candidates=min_candidates,
                                                 max_waves=max_waves)
            model, keep, st_f = self.filter_run(model)
            model = model[keep == 1]
            log.append({"depth": depth, "expand": st_e, "filter": st_f, "patches": len(model)})
            ncc = np.float32(ncc - np.float32(0.05))
            before = np.float32(before - np.float32(0.05))
            cthr = 2
            depth += 1
        return model, log

    def loop_fetch(self, n: int) -> np.ndarray:
        """pmvs_loop_fetch: the n-patch result of the last run_loop(fetch=False), device to host."""
        out = np.empty(n, PATCH_DTYPE)
        _check(self.lib.pmvs_loop_fetch(self.handle, _ptr(out), n))
        return out

    def loop_hash(self) -> int:
        """pmvs_loop_hash: 64-bit digest of the last run_loop result still on the device."""
        h = C.c_uint64(0)
        _check(self.lib.pmvs_loop_hash(self.handle, C.byref(h)))
        return int(h.value)

    def patch_colors(self, coords: np.ndarray, images) -> np.ndarray:
        """writePLY colour mode 0 for patches (coords [n,4], images: list of view-index lists)."""
        coords = np.ascontiguousarray(coords, np.float32).reshape(-1, 4)
        nimg = np.array([len(x) for x in images], np.int32)
        flat = np.array([v for x in images for v in x] or [0], np.int32)
        out = np.zeros((len(coords), 3), np.int32)
        _check(self.lib.pmvs_patch_colors(self.handle, len(coords), _ptr(coords), _ptr(nimg), _ptr(flat), _ptr(out)))
        return out

    def sync(self):
        st = Stats()
        _check(self.lib.pmvs_scene_sync(self.handle, C.byref(st)))
        return st.as_dict()


def points_flat(points):
    """Per-view feature points -> (flat POINT_DTYPE array, per-view counts)."""
    parts = []
    for pv in points:
        if isinstance(pv, np.ndarray) and pv.dtype == POINT_DTYPE:
            parts.append(pv)
            continue
        a = np.asarray(pv, np.float32).reshape(-1, 4)
        r = np.zeros(len(a), POINT_DTYPE)
        r["x"], r["y"], r["response"], r["type"] = a[:, 0], a[:, 1], a[:, 2], a[:, 3].astype(np.int32)
        parts.append(r)
    npts = np.array([len(p) for p in parts], np.int32)
    flat = np.concatenate(parts) if parts and npts.sum() else np.zeros(1, POINT_DTYPE)
    return np.ascontiguousarray(flat), npts


def selftest_math(op: int, x: np.ndarray, device: int = 0) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float64)
    out = np.zeros_like(x)
    _check(load_library().pmvs_selftest_math(device, op, _ptr(x), _ptr(out), len(x)))
    return out


def selftest_lls(systems, device: int = 0) -> np.ndarray:
    """Device lls (filterQuad's least squares) on a list of (A [n, 5], b [n]) systems: x [k, 5]."""
    A = np.ascontiguousarray(np.concatenate([np.asarray(a, np.float32).reshape(-1, 5) for a, _ in systems]))
    b = np.ascontiguousarray(np.concatenate([np.asarray(v, np.float32).reshape(-1) for _, v in systems]))
    off = np.zeros(len(systems) + 1, np.int32)
    off[1:] = np.cumsum([len(v) for _, v in systems])
    x = np.zeros((len(systems), 5), np.float32)
    _check(load_library().pmvs_selftest_lls(device, _ptr(A), _ptr(b), _ptr(off), len(systems), _ptr(x)))
    return x


def selftest_bobyqa(kind: int, x0: np.ndarray, mode: int = 0, maxeval: int = 1000, device: int = 0):
    x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 3)
    out = np.zeros((len(x0), 6), np.float64)
    ms = C.c_double()
    _check(load_library().pmvs_selftest_bobyqa(device, mode, kind, _ptr(x0), len(x0), maxeval, _ptr(out), C.byref(ms)))
    return out, ms.value


# ---------------------------------------------------------------------------------- pmvs2 I/O
def camera_load(path: str) -> np.ndarray:
    """CONTOUR/CONTOUR2/CONTOUR3 txt -> level-0 3x4 projection (pmvs_camera_load)."""
    out = np.zeros(12, np.float32)
    _check(load_library().pmvs_camera_load(path.encode(), _ptr(out)))
    return out.reshape(3, 4)


def ppm_load(path: str) -> np.ndarray:
    lib = load_library()
    w, h = C.c_int32(), C.c_int32()
    _check(lib.pmvs_ppm_load(path.encode(), C.byref(w), C.byref(h), None))
    img = np.zeros((h.value, w.value, 3), np.uint8)
    _check(lib.pmvs_ppm_load(path.encode(), C.byref(w), C.byref(h), _ptr(img)))
    return img


def image_load(path: str) -> np.ndarray:
    """CImage::readAnyImage: PPM or JPEG -> uint8 [H, W, 3] (pmvs_image_load)."""
    lib = load_library()
    w, h = C.c_int32(), C.c_int32()
    _check(lib.pmvs_image_load(path.encode(), C.byref(w), C.byref(h), None))
    img = np.zeros((h.value, w.value, 3), np.uint8)
    _check(lib.pmvs_image_load(path.encode(), C.byref(w), C.byref(h), _ptr(img)))
    return img


def mask_load(path: str) -> np.ndarray:
    """Binary PGM (P5) / PBM (P4) mask or edge image -> uint8 [H, W] (pmvs_pnm_mask_load)."""
    lib = load_library()
    w, h = C.c_int32(), C.c_int32()
    _check(lib.pmvs_pnm_mask_load(path.encode(), C.byref(w), C.byref(h), None))
    m = np.zeros((h.value, w.value), np.uint8)
    _check(lib.pmvs_pnm_mask_load(path.encode(), C.byref(w), C.byref(h), _ptr(m)))
    return m


def set_edge(rgb: np.ndarray, threshold: float) -> np.ndarray:
    """CImage::setEdge (option setEdge): edge map of a level-0 image (pmvs_set_edge)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    out = np.zeros(rgb.shape[:2], np.uint8)
    _check(load_library().pmvs_set_edge(_ptr(rgb), rgb.shape[1], rgb.shape[0], float(threshold), _ptr(out)))
    return out


def options_load(prefix: str, option_file: str) -> dict:
    """pmvs2 option file (+ vis.dat / bimages.dat) -> dict (pmvs_options_load)."""
    lib = load_library()
    p = C.POINTER(Options)()
    _check(lib.pmvs_options_load(prefix.encode(), option_file.encode(), C.byref(p)))
    o = p.contents
    d = {k: getattr(o, k) for k, _ in Options._fields_[:17]}
    num = o.num_timages + o.num_oimages
    d["timages"] = [o.timages[i] for i in range(o.num_timages)]
    d["oimages"] = [o.oimages[i] for i in range(o.num_oimages)]
    d["bindexes"] = [o.bindexes[i] for i in range(o.num_bindexes)]
    off = [o.visdata2_offsets[i] for i in range(num + 1)]
    d["visdata2"] = [[o.visdata2[k] for k in range(off[r], off[r + 1])] for r in range(num)]
    lib.pmvs_options_free(p)
    return d


def _patch_arrays(fields, images, vimages):
    fields = np.ascontiguousarray(fields, np.float32).reshape(-1, 11)
    nimg = np.array([len(x) for x in images], np.int32)
    nv = np.array([len(x) for x in vimages], np.int32)
    ids = np.array([v for x in images for v in x] or [0], np.int32)
    vids = np.array([v for x in vimages for v in x] or [0], np.int32)
    return fields, nimg, ids, nv, vids


def write_patches(path: str, fields, images, vimages):
    f, nimg, ids, nv, vids = _patch_arrays(fields, images, vimages)
    _check(load_library().pmvs_write_patches(path.encode(), len(f), _ptr(f), _ptr(nimg), _ptr(ids), _ptr(nv),
                                             _ptr(vids)))


def write_pset(path: str, fields):
    f = np.ascontiguousarray(fields, np.float32).reshape(-1, 11)
    _check(load_library().pmvs_write_pset(path.encode(), len(f), _ptr(f)))


def write_ply(path: str, fields, colors):
    f = np.ascontiguousarray(fields, np.float32).reshape(-1, 11)
    c = np.ascontiguousarray(colors, np.int32).reshape(-1, 3)
    _check(load_library().pmvs_write_ply(path.encode(), len(f), _ptr(f), _ptr(c)))


def patches_from_refined(refined: np.ndarray) -> np.ndarray:
    """Accepted pmvs_refined records -> pmvs_patch records (the CPatch fields a filter pass reads)."""
    acc = refined[refined["status"] == ACCEPTED]
    p = np.zeros(len(acc), PATCH_DTYPE)
    for f in ("coord", "normal", "ncc", "dscale", "ascale", "tmp", "timages", "num_images", "images"):
        p[f] = acc[f]
    p["grids"] = grid16(acc["grids"])
    return p


def grid16(g):
    """Cell coordinates as pmvs_patch stores them (int16): values outside [-32767, 32767] -- only
    projections far outside the image, so outside every cell grid -- become -32768 (pmvs_layout.h)."""
    g = np.asarray(g, np.int64)
    return np.where((g < -32767) | (g > 32767), -32768, g).astype(np.int16)


def device_count() -> int:
    return int(load_library().pmvs_device_count())


# ---------------------------------------------------------------------------------- synthetic data
def synth_params(num_views: int, width: int, height: int, num_targets: Optional[int] = None,
                 supersample: int = 2, level: int = 1, seed: int = 0x504D5653,
                 ring_radius: float = 4.0, height_offset: float = 0.3, focal_scale: float = 1.16,
                 arc_step_deg: Optional[float] = None, hard: bool = False) -> SynthParams:
    p = SynthParams()
    p.num_views = num_views
    p.num_targets = num_views if num_targets is None else num_targets
    p.width, p.height = width, height
    p.supersample = supersample
    p.level = level
    p.seed = seed
    p.ring_radius, p.height_offset, p.focal_scale = ring_radius, height_offset, focal_scale
    # cameras every min(360/V, 15) degrees: a full ring for V >= 24, an arc otherwise
    p.arc_step_deg = min(360.0 / num_views, 15.0) if arc_step_deg is None else arc_step_deg
    for k, v in (HARD if hard else {}).items():
        setattr(p, k, v)
    return p


def synth_ring(p: SynthParams, nthreads: int = 8, render: bool = True):
    """(rgb of the rendered views -- all, or p.render_count from p.render_first --, every view's projection)."""
    lib = load_library()
    proj = np.zeros((p.num_views, 3, 4), np.float32)
    count = p.render_count if p.render_count > 0 else p.num_views
    rgb = np.zeros((count, p.height, p.width, 3), np.uint8) if render else None
    _check(lib.pmvs_synth_ring(C.byref(p), _ptr(rgb), _ptr(proj), nthreads))
    return rgb, proj


def synth_candidates(p: SynthParams, proj: np.ndarray, n: int, seed: int = 0x5EED,
                     depth_sigma_px: float = 1.0, max_tilt_deg: float = 10.0) -> np.ndarray:
    lib = load_library()
    out = np.zeros(n, CANDIDATE_DTYPE)
    proj = np.ascontiguousarray(proj, np.float32)
    _check(lib.pmvs_synth_candidates(C.byref(p), _ptr(proj), n, seed, depth_sigma_px, max_tilt_deg, _ptr(out)))
    return out


def synth_scene(num_views: int, width: int, height: int, level: int = 1, num_targets: Optional[int] = None,
                supersample: int = 2, nthreads: int = 8, seed: int = 0x504D5653, hard: bool = False,
                arc_step_deg: Optional[float] = None, **opts) -> SceneInputs:
    p = synth_params(num_views, width, height, num_targets=num_targets, supersample=supersample, level=level,
                     seed=seed, hard=hard, arc_step_deg=arc_step_deg)
    rgb, proj = synth_ring(p, nthreads=nthreads)
    return SceneInputs(images=[rgb[i] for i in range(num_views)], projections=proj,
                       num_targets=p.num_targets, level=level, **opts), p


class ThreadExchange:
    """In-process all-gather among `world` threads (pmvs_thread_exchange): scene r of a group uses
    set_shard(r, world, *group.endpoint(r)).  Used to run several sharded scenes on one GPU."""

    def __init__(self, world: int):
        self.lib = load_library()
        self.world = world
        self.handle = self.lib.pmvs_thread_exchange_create(world)
        if not self.handle:
            raise PmvsError("pmvs_thread_exchange_create failed")

    def endpoint(self, rank: int):
        fn = C.cast(self.lib.pmvs_thread_allgather, C.c_void_p).value
        return fn, self.lib.pmvs_thread_exchange_ctx(self.handle, rank)

    def close(self):
        if self.handle:
            self.lib.pmvs_thread_exchange_destroy(self.handle)
            self.handle = None


class RcclExchange:
    """Native RCCL communicator of the sharded expansion (pmvs_rccl_*): one process per GPU; the
    per-wave records go device to device on the scene's stream.  Rank 0 creates the 128-byte id
    (unique_id()) and every rank receives it (e.g. torch.distributed.broadcast_object_list)."""

    def __init__(self, rank: int, world: int, uid: bytes, device: int = 0):
        self.lib = load_library()
        self.rank, self.world = rank, world
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(self.lib.pmvs_rccl_create(device, rank, world, buf, C.byref(h)))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        _check(load_library().pmvs_rccl_unique_id(buf))
        return bytes(buf)

    def allgather(self, data: bytes) -> bytes:
        n = len(data)
        out = (C.c_uint8 * (n * self.world))()
        src = (C.c_uint8 * max(1, n)).from_buffer_copy(data if n else b"\0")
        if self.lib.pmvs_rccl_allgather(self.handle, src, n, out) != 0:
            raise PmvsError("pmvs_rccl_allgather failed")
        return bytes(out)

    def attach(self, scene: "Scene"):
        _check(self.lib.pmvs_scene_set_shard_rccl(scene.handle, self.rank, self.world, self.handle))

    def attach_cluster(self, scene: "Scene", image_ids):
        """The scene is this rank's CMVS cluster; its boundary patches go device to device over RCCL."""
        ids = np.ascontiguousarray(image_ids, np.int32)
        scene._cluster_keep = (None, ids)
        _check(self.lib.pmvs_scene_set_cluster_rccl(scene.handle, self.rank, self.world, _ptr(ids), self.handle))

    def close(self):
        if self.handle:
            self.lib.pmvs_rccl_destroy(self.handle)
            self.handle = None


class DistExchange:
    """pmvs_allgather_fn over torch.distributed: one process per GPU (RCCL over xGMI when the
    process group's backend is nccl; gloo on CPUs).  The host buffer of each expansion wave is
    staged through a device tensor for RCCL.  Keep the object alive while the scene uses it."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.dist, self.torch, self.group = dist, torch, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        backend = dist.get_backend(group)
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu"))
        self.error = None
        self.fn = ALLGATHER_FN(self._allgather)

    def _allgather(self, ctx, send, nbytes, recv):
        try:
            torch = self.torch
            src = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(nbytes,))
            t = torch.from_numpy(src.copy()).to(self.device)
            if self.device.type == "cpu":  # gloo: list form
                parts = [torch.empty_like(t) for _ in range(self.world)]
                self.dist.all_gather(parts, t, group=self.group)
                res = torch.cat(parts).numpy()
            else:
                out = torch.empty(nbytes * self.world, dtype=torch.uint8, device=self.device)
                self.dist.all_gather_into_tensor(out, t, group=self.group)
                res = out.cpu().numpy()
            C.memmove(recv, res.ctypes.data, nbytes * self.world)
            return 0
        except Exception as e:  # reported by pmvs_expand_run as a failed exchange
            self.error = e
            return -1

    def attach(self, scene: "Scene"):
        scene.set_shard(self.rank, self.world, self.fn, None)
