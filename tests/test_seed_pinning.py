"""CPU tests of the seed-phase oracle (oracle/seed_oracle.h, CSeed seed.cpp:11-414).

Reference pinning (tests/golden/seeds.npz, made by tests/golden/make_golden.py from oracle/_ref):
Image::setF, Image::computeEPD (camera.hpp:119-151) and the CSeed::unproject triangulation
(seed.cpp:340-384) evaluated with the reference's own CCamera and numeric headers, for feature
point pairs of the golden scenes.  The oracle's seed patches are a regression vector (the full
CSeed needs CFindMatch / COptim, which do not build here: nlopt is absent)."""
import os

import numpy as np
import pytest

from pmvs_cases import bits

HERE = os.path.dirname(os.path.abspath(__file__))
SCENES = {"c1": (3, 640, 480, 2, 4), "ring8": (8, 320, 240, 1, 2)}


@pytest.fixture(scope="module")
def goldens():
    return dict(np.load(os.path.join(HERE, "golden", "seeds.npz"))), dict(np.load(os.path.join(HERE, "golden",
                                                                                                 "features.npz")))


def _scene(name, oracle_mod):
    import pmvs_amd as P
    views, w, h, level, csize = SCENES[name]
    inp, p = P.synth_scene(views, w, h, level=level, csize=csize, supersample=2)
    return inp, oracle_mod.OracleScene(inp)


@pytest.mark.parametrize("name", list(SCENES))
def test_seed_geometry_matches_reference(name, goldens, oracle_mod, product_lib):
    """oracle setF / computeEPD / unproject == the reference headers, bit for bit."""
    g, _ = goldens
    inp, o = _scene(name, oracle_mod)
    xy = g[f"{name}_xy"]
    k = 0
    for pi, (i0, i1) in enumerate(g[f"{name}_pairs"]):
        n = int(g[f"{name}_pair_len"][pi])
        F, epd, co = o.seed_geometry(int(i0), int(i1), xy[k:k + n, 0], xy[k:k + n, 1])
        assert np.array_equal(bits(F), bits(g[f"{name}_ref_F"][pi])), (i0, i1, "F")
        assert np.array_equal(bits(epd), bits(g[f"{name}_ref_epd"][k:k + n])), (i0, i1, "epd")
        assert np.array_equal(bits(co), bits(g[f"{name}_ref_coords"][k:k + n])), (i0, i1, "unproject")
        k += n
    o.close()


@pytest.mark.parametrize("name", list(SCENES))
def test_seed_run_golden(name, goldens, oracle_mod, product_lib):
    """CSeed::run (CPU 1) on the reference-detected features == the committed seed patches."""
    g, feats = goldens
    inp, o = _scene(name, oracle_mod)
    off = feats[f"{name}_offsets"]
    pts = [feats[f"{name}_points"][off[v]:off[v + 1]] for v in range(len(inp.images))]
    seeds, st = o.seed_run(pts)
    o.close()
    assert [st[k] for k in ("trial", "pass", "fail0", "fail1")] == g[f"{name}_seed_stats"].tolist()
    assert len(seeds) == len(g[f"{name}_seeds"]) > 0
    assert seeds.tobytes() == g[f"{name}_seeds"].tobytes()


def test_seed_geometry_live_reference(oracle_mod, product_lib, tmp_path):
    """Random point pairs (not only features) against the reference headers, when oracle/_ref is
    built (build container only)."""
    R = oracle_mod.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (reference absent)")
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden as M
    inp, o = _scene("ring8", oracle_mod)
    rng = np.random.default_rng(5)
    for i0, i1 in [(2, 3), (5, 1), (7, 0)]:
        xy0 = rng.uniform(0, 159, (500, 2)).astype(np.float32)
        xy1 = rng.uniform(0, 119, (500, 2)).astype(np.float32)
        F, epd, co = o.seed_geometry(i0, i1, xy0, xy1)
        rF, repd, rco = M.ref_seed_geometry(inp.projections, 4, 1, i0, i1, xy0, xy1)
        assert np.array_equal(bits(F), bits(rF))
        assert np.array_equal(bits(epd), bits(repd))
        assert np.array_equal(bits(co), bits(rco))
    o.close()


def test_seed_candidates_sorted(goldens, oracle_mod, product_lib):
    """Candidate lists: ascending _response, ties in collection order, every EPD < 2 px."""
    g, feats = goldens
    inp, o = _scene("ring8", oracle_mod)
    off = feats["ring8_offsets"]
    pts = [feats["ring8_points"][off[v]:off[v + 1]] for v in range(len(inp.images))]
    total = 0
    for pid in range(0, len(pts[0]), 7):
        oi, of = o.seed_candidates(pts, 0, pid)
        total += len(oi)
        assert np.all(np.diff(of[:, 4]) >= 0)
        for (view, q, cell), f in zip(oi, of):
            _, epd, _ = o.seed_geometry(0, int(view), pts[0][pid:pid + 1, :2], pts[view][q:q + 1, :2])
            assert epd[0] < 2.0
            assert pts[view][q, 3] == pts[0][pid, 3]
    assert total > 0
    o.close()
