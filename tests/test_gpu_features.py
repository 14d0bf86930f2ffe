"""Feature detection: pmvs_detect_features -- CHarris + CDifferenceOfGaussians
as HIP kernels (cmvs-pmvs_amd/csrc/pmvs_features.hip) -- against the REFERENCE's own detectors.

The reference's harris.cpp / dog.cpp / detector.cpp / point.cpp compile unmodified in this image,
so they are the oracle here (oracle/_ref ref_detect_features, detectFeatures.cpp's calls and
ordering).  tests/golden/features.npz holds their output on every view of the two golden scenes;
the masked / edged cases are compared with the live reference library.  Bar: bit-exact points
(coordinates, responses, types) in the reference's order."""
import os

import numpy as np
import pytest

from pmvs_cases import bits

GOLD = os.path.join(os.path.dirname(__file__), "golden", "features.npz")
SCENES = {"c1": (3, 640, 480, 2, 4), "ring8": (8, 320, 240, 1, 2)}  # as tests/golden/make_golden.py


def _as_rows(points):
    return np.stack([points["x"], points["y"], points["response"], points["type"].astype(np.float32)], 1)


def test_golden_features_match_live_reference(oracle_mod):
    """The committed fixture is what the reference detectors produce (pins the fixture)."""
    import pmvs_amd as P
    if oracle_mod.ref_lib() is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    g = dict(np.load(GOLD))
    for name, (views, w, h, level, csize) in SCENES.items():
        inp, _ = P.synth_scene(views, w, h, level=level, csize=csize, supersample=2)
        o = oracle_mod.OracleScene(inp)
        off = g[f"{name}_offsets"]
        for v in range(views):
            f = oracle_mod.ref_detect_features(o.get_level(v, level))
            assert np.array_equal(bits(f), bits(g[f"{name}_points"][off[v]:off[v + 1]])), (name, v)
        o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES))
def test_features_match_reference_golden(gpu_available, name):
    import pmvs_amd as P
    views, w, h, level, csize = SCENES[name]
    g = dict(np.load(GOLD))
    inp, _ = P.synth_scene(views, w, h, level=level, csize=csize, supersample=2)
    s = P.Scene(inp)
    off = g[f"{name}_offsets"]
    for v in range(views):
        got = _as_rows(s.detect_features(v, 16))
        exp = g[f"{name}_points"][off[v]:off[v + 1]]
        assert got.shape == exp.shape, (name, v, got.shape, exp.shape)
        assert np.array_equal(bits(got), bits(exp)), (name, v)
    s.close()


def _binary_levels(m, level, thresh):
    """The scene's binary pyramid (pmvs_api.cpp build_binary: level 0 = m > thresh; then a
    level-l pixel is set when any of its 2x2 parents is, CImage::buildMask image.cpp:327-361)."""
    b = np.where(m > thresh, 255, 0).astype(np.uint8)
    for _ in range(level):
        H, W = b.shape[0] // 2, b.shape[1] // 2
        ys0, xs0 = 2 * np.arange(H), 2 * np.arange(W)
        ys1, xs1 = np.minimum(b.shape[0] - 1, ys0 + 1), np.minimum(b.shape[1] - 1, xs0 + 1)
        any_ = (b[np.ix_(ys0, xs0)] | b[np.ix_(ys0, xs1)] | b[np.ix_(ys1, xs0)] | b[np.ix_(ys1, xs1)]) > 0
        b = np.where(any_, 255, 0).astype(np.uint8)
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("use_mask,use_edge", [(True, False), (False, True), (True, True)])
def test_features_with_masks_match_live_reference(gpu_available, oracle_mod, use_mask, use_edge):
    import pmvs_amd as P
    from test_gpu_parity_matrix import blob_masks
    if oracle_mod.ref_lib() is None:
        pytest.fail("oracle/_ref missing: build it in the build container (make -C oracle) so it ships with the tree")
    V, w, h, level = 4, 480, 360, 1
    inp, _ = P.synth_scene(V, w, h, level=level, supersample=2)
    if use_mask:
        inp.masks = blob_masks(V, h, w, 5, keep=0.8)
    if use_edge:
        inp.edges = blob_masks(V, h, w, 6, keep=0.85)
    s = P.Scene(inp)
    for v in range(V):
        got = _as_rows(s.detect_features(v, 16))
        img = s.get_level(v, level)
        m = _binary_levels(inp.masks[v], level, 127) if use_mask else None
        e = _binary_levels(inp.edges[v], level, 1) if use_edge else None
        exp = oracle_mod.ref_detect_features(img, m, e, fcsize=16)
        assert got.shape == exp.shape, (v, got.shape, exp.shape)
        assert np.array_equal(bits(got), bits(exp)), v
    s.close()


@pytest.mark.gpu
def test_features_large_view_matches_reference(gpu_available, oracle_mod):
    """One 1920x1080 view at level 0 (the C2/C3 image class; thousands of blocks)."""
    import pmvs_amd as P
    if oracle_mod.ref_lib() is None:
        pytest.fail("oracle/_ref missing")
    inp, _ = P.synth_scene(3, 1920, 1080, level=0, supersample=1)
    s = P.Scene(inp)
    got = _as_rows(s.detect_features(0, 16))
    exp = oracle_mod.ref_detect_features(s.get_level(0, 0), fcsize=16)
    s.close()
    assert len(exp) > 1000
    assert np.array_equal(bits(got), bits(exp))
