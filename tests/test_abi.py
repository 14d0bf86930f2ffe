"""CPU tests of the drop-in boundary: libpmvs_amd.so loads without a GPU, exports every entry
point include/pmvs_amd.h declares, the Python mirror's record layouts equal the C compiler's,
and compute entry points fail loudly (status, message) when no HIP device is present --
there is no CPU fallback behind the ABI."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pmvs_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pmvs_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pmvs_refine_batch" in syms and "pmvs_scene_create" in syms
    assert len(syms) >= 15


def test_library_exports_every_declared_symbol(product_lib):
    out = subprocess.run(["nm", "-D", "--defined-only",
                          os.path.join(ROOT, "cmvs-pmvs_amd", "libpmvs_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    import pmvs_amd as P
    assert set(P.EXPORTS) <= set(declared_symbols())


def test_python_mirror_layout_matches_c(tmp_path):
    exe = tmp_path / "abi_layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "csrc", "abi_layout.c"), "-o", str(exe)], check=True)
    c = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        k, *rest = line.split()
        c[k if rest[0] != "sizeof" else k + ".sizeof"] = int(rest[-1])
    import pmvs_amd as P
    np_types = {"pmvs_candidate": P.CANDIDATE_DTYPE, "pmvs_refined": P.REFINED_DTYPE,
                "pmvs_eval_query": P.EVAL_QUERY_DTYPE, "pmvs_tex_query": P.TEX_QUERY_DTYPE,
                "pmvs_patch": P.PATCH_DTYPE, "pmvs_point": P.POINT_DTYPE}
    for name, dt in np_types.items():
        assert dt.itemsize == c[name + ".sizeof"], name
        for f in dt.names:
            key = f"{name}.{f}"
            if key in c:
                assert dt.fields[f][1] == c[key], key
    ct_types = {"pmvs_view_desc": P.ViewDesc, "pmvs_scene_desc": P.SceneDesc, "pmvs_stats": P.Stats,
                "pmvs_synth_params": P.SynthParams, "pmvs_filter_stats": P.FilterStats, "pmvs_options": P.Options,
                "pmvs_expand_stats": P.ExpandStats, "pmvs_loop_iter": P.LoopIter,
                "pmvs_seed_stats": P.SeedStats}
    for name, T in ct_types.items():
        assert C.sizeof(T) == c[name + ".sizeof"], name
        for f, _ in T._fields_:
            key = f"{name}.{f}"
            if key in c:
                assert getattr(T, f).offset == c[key], key


def test_no_device_fails_loudly(product_lib):
    """On a host without a HIP device the compute entry points return an error status with a
    message; nothing silently computes on the CPU."""
    import pmvs_amd as P
    if P.device_count() > 0:
        pytest.skip("a HIP device is visible")
    inp, p = P.synth_scene(3, 64, 48, level=1)
    with pytest.raises(P.PmvsError):
        P.Scene(inp)
    with pytest.raises(P.PmvsError):
        P.selftest_math(0, np.ones(4))


def test_invalid_arguments_rejected(product_lib):
    lib = product_lib
    h = C.c_void_p()
    assert lib.pmvs_scene_create(None, 0, C.byref(h)) != 0
    assert lib.pmvs_last_error()
    assert lib.pmvs_refine_batch(None, None, 0, None, None) != 0


def test_cell_index_range_rejected(product_lib):
    """Target cells are indexed with 32-bit ints (pgrids, commit records): a scene whose target
    cells at its level exceed 2^31 - 1 (64 targets of 8192x4320 at csize 1) is rejected as
    PMVS_EUNSUPPORTED before anything is allocated (advice r01, low)."""
    import pmvs_amd as P
    lib = product_lib
    nv = 64
    views = (P.ViewDesc * nv)()
    for v in views:
        v.width, v.height = 8192, 4320
    off = (C.c_int32 * (nv + 1))()
    d = P.SceneDesc(num_views=nv, num_targets=nv, level=0, csize=1, wsize=7, min_image_num=3, threshold=0.7,
                    max_angle=10.0, quad_threshold=2.0, sequence=-1, visdata2_offsets=C.cast(off, C.c_void_p),
                    views=views)
    h = C.c_void_p()
    assert lib.pmvs_scene_create(C.byref(d), 0, C.byref(h)) == 4  # PMVS_EUNSUPPORTED
    assert b"target cells" in lib.pmvs_last_error()
