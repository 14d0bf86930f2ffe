"""GPU parity: the HIP path (libpmvs_amd.so via the C-ABI) against the CPU oracle
(oracle/liboracle.so) on identical seeded inputs.  Integer/index outputs and every float the
reference computes in float are compared BIT-EXACTLY (np.array_equal on the raw bits)."""
import numpy as np
import pytest

from conftest import small_scene

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


@pytest.fixture(scope="module")
def scenes(gpu_available, oracle_mod):
    import pmvs_amd as P
    inp, p = small_scene(8, 480, 360, level=1)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    yield inp, p, g, o
    g.close()
    o.close()


def test_pyramid_levels_bit_exact(scenes):
    inp, p, g, o = scenes
    for v in range(len(inp.images)):
        for lv in range(inp.level + 3):
            a = g.get_level(v, lv)
            b = o.get_level(v, lv)
            assert a.shape == b.shape
            assert np.array_equal(a, b), (v, lv, int((a != b).sum()))


def test_grab_tex_bit_exact(scenes):
    import pmvs_amd as P
    inp, p, g, o = scenes
    cands = P.synth_candidates(p, inp.projections, 300, seed=11)
    q = np.zeros(len(cands) * 3, P.TEX_QUERY_DTYPE)
    k = 0
    for c in cands:
        ref = int(c["images"][0])
        px, py = o.paxes(ref, c["coord"], c["normal"])
        for view in (ref, int(c["images"][1]), (ref + 3) % len(inp.images)):
            q[k]["coord"] = c["coord"]
            q[k]["pxaxis"] = px
            q[k]["pyaxis"] = py
            q[k]["normal"] = c["normal"]
            q[k]["view"] = view
            q[k]["normalize"] = k % 2
            k += 1
    tg, vg = g.grab_tex(q)
    to, vo = o.grab_tex(q)
    assert np.array_equal(vg, vo)
    assert vo.sum() > len(q) // 3
    assert np.array_equal(bits(tg), bits(to))


def test_incc_eval_bit_exact(scenes):
    import pmvs_amd as P
    inp, p, g, o = scenes
    cands = P.synth_candidates(p, inp.projections, 200, seed=12)
    rng = np.random.default_rng(3)
    q = np.zeros(len(cands) * 4, P.EVAL_QUERY_DTYPE)
    V = len(inp.images)
    for i, c in enumerate(cands):
        ref = int(c["images"][0])
        others = [v for v in np.argsort(np.abs(np.arange(V) - ref)) if v != ref][:5]
        for j in range(4):
            r = q[4 * i + j]
            r["coord"], r["normal"] = c["coord"], c["normal"]
            r["dscale"] = 0.002 * (1 + j)
            r["num_images"] = 6
            r["images"][:6] = [ref] + list(others)
            r["x"] = rng.normal(0, [2.0, 3.0, 3.0]) if j else [0.0, 0.0, 0.0]
    fg, st = g.incc_eval(q)
    fo = o.incc_eval(q)
    assert (fo < 2.0).sum() > len(q) // 4
    assert np.array_equal(bits(fg), bits(fo)), np.flatnonzero(bits(fg) != bits(fo))[:10]
    assert st["evals"] == len(q)


def compare_refined(rg, ro):
    assert np.array_equal(rg["status"], ro["status"])
    acc = ro["status"] == 0
    for f in ("refine_code", "evals", "num_images", "timages"):
        assert np.array_equal(rg[f][acc], ro[f][acc]), f
    for f in ("coord", "normal", "ncc", "dscale", "ascale", "tmp"):
        assert np.array_equal(bits(rg[f][acc]), bits(ro[f][acc])), f
    for i in np.flatnonzero(acc):
        n = ro["num_images"][i]
        assert np.array_equal(rg["images"][i][:n], ro["images"][i][:n])
        assert np.array_equal(rg["grids"][i][:n], ro["grids"][i][:n])


def test_refine_batch_bit_exact(scenes):
    import pmvs_amd as P
    inp, p, g, o = scenes
    cands = P.synth_candidates(p, inp.projections, 400, seed=13)
    rg, sg = g.refine_batch(cands)
    ro, so = o.refine_batch(cands, nthreads=8)
    assert so["accepted"] > 100
    compare_refined(rg, ro)
    for k in ("accepted", "fail_pre", "fail_post", "refine_failed", "evals", "tex_valid"):
        assert sg[k] == so[k], k


REFINE_CONFIGS = [300000, 300004, 300008, 1206, 2408, 164011, 164021, 164041, 148041, 132022, 132042, 116042, 202032, 224016, 225016, 226014, 227012, 228010, 245016, 246014, 248010]


@pytest.mark.parametrize("config", REFINE_CONFIGS)
def test_refine_configs_bit_exact(scenes, monkeypatch, config):
    """Every refine-kernel layout (PMVS_REFINE_CONFIG: the wavefront form's texture slots * 100 +
    chains, the workgroup form's 100000 + chains * 1000 + optimizer wavefronts * 10 + workgroups per
    CU) gives the oracle's records, for a batch that fills the chip and for a 5-candidate one."""
    import pmvs_amd as P
    inp, p, g, o = scenes
    monkeypatch.setenv("PMVS_REFINE_CONFIG", str(config))
    gc = P.Scene(inp)
    try:
        for n, seed in ((3000, 21), (5, 22)):
            cands = P.synth_candidates(p, inp.projections, n, seed=seed)
            rg, sg = gc.refine_batch(cands)
            ro, so = o.refine_batch(cands, nthreads=8)
            compare_refined(rg, ro)
            for k in ("accepted", "fail_pre", "fail_post", "refine_failed", "evals", "tex_valid"):
                assert sg[k] == so[k], (n, k)
    finally:
        gc.close()


def test_full_size_c2_batch_parity(gpu_available, oracle_mod):
    """BASELINE configs[1] at full size (8 views 1920x1080, level 1, 100k seed candidates):
    every record of the HIP path equals the oracle's."""
    import pmvs_amd as P
    inp, p = P.synth_scene(8, 1920, 1080, level=1, supersample=2, nthreads=16)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    cands = P.synth_candidates(p, inp.projections, 100000, seed=0x5EED)
    rg, sg = g.refine_batch(cands)
    ro, so = o.refine_batch(cands, nthreads=16)
    g.close()
    o.close()
    bad = np.flatnonzero(rg["status"] != ro["status"])
    assert len(bad) == 0, (len(bad), bad[:10])
    compare_refined(rg, ro)
    for k in ("accepted", "fail_pre", "fail_post", "refine_failed", "evals", "tex_valid"):
        assert sg[k] == so[k], k


def _np_get_color(img, x, y):
    """CImage::getColor bilinear (image.hpp:435-476) in IEEE float32, same operation order."""
    f32 = np.float32
    lx, ly = int(x), int(y)
    dx1 = f32(x) - f32(lx); dx0 = f32(1) - dx1
    dy1 = f32(y) - f32(ly); dy0 = f32(1) - dy1
    f00, f01, f10, f11 = dx0 * dy0, dx0 * dy1, dx1 * dy0, dx1 * dy1
    a0, a1 = img[ly, lx].astype(np.float32), img[ly, lx + 1].astype(np.float32)
    b0, b1 = img[ly + 1, lx].astype(np.float32), img[ly + 1, lx + 1].astype(np.float32)
    out = np.zeros(3, np.float32)
    out = out + (a0 * f00 + b0 * f01)
    out = out + (a1 * f10 + b1 * f11)
    return out


def test_patch_colors_match_reference_formula(scenes):
    """writePLY colour mode 0 on the device == the reference formula evaluated on the oracle's
    pyramid and projections (patchOrganizerS.cpp:716-731)."""
    import pmvs_amd as P
    inp, p, g, o = scenes
    cands = P.synth_candidates(p, inp.projections, 200, seed=21)
    images = [list(map(int, c["images"][:c["num_images"]])) for c in cands]
    got = g.patch_colors(cands["coord"], images)
    lv = inp.level
    pyr = {v: o.get_level(v, lv) for v in range(len(inp.images))}
    for i, c in enumerate(cands):
        acc = np.zeros(3, np.float32)
        for v in images[i]:
            ic = o.project(v, lv, c["coord"][None, :])[0]
            acc = acc + _np_get_color(pyr[v], ic[0], ic[1])
        m = acc / np.float32(len(images[i]))
        exp = [min(255, int(np.floor(np.float64(np.float32(m[j] + np.float32(0.5)))))) for j in range(3)]
        assert list(got[i]) == exp, i
