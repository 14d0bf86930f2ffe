"""GPU parity of the seed phase (pmvs_seed_run, CSeed seed.cpp:11-414): epipolar candidates,
triangulation and the _response order on the device, speculative batched refinement, and the
host replay of the reference's sequential control -- against the CPU oracle's CSeed restatement
(oracle/seed_oracle.h, CPU 1 order), bit for bit, for every batch size and across the option
space.  The end-to-end case runs features -> seeds -> the expand/filter loop (C1)."""
import numpy as np
import pytest

from test_gpu_parity_matrix import CONFIGS, build

pytestmark = pytest.mark.gpu

SEED_FIELDS = ("coord", "normal", "ncc", "dscale", "ascale", "tmp", "timages", "num_images", "images", "grids")


def features(g, inp):
    return [g.detect_features(v) for v in range(len(inp.images))]


def same_seeds(a, b):
    assert len(a) == len(b)
    for f in SEED_FIELDS:
        assert a[f].tobytes() == b[f].tobytes(), f


def run_pair(inp, batch=0):
    import pmvs_amd as P
    import pyoracle as O
    g = P.Scene(inp)
    o = O.OracleScene(inp)
    pts = features(g, inp)
    sg, stg = g.seed_run(pts, batch=batch)
    so, sto = o.seed_run(pts)
    return g, o, pts, sg, stg, so, sto


@pytest.mark.parametrize("name,views,w,h,level,csize", [("c1", 3, 640, 480, 2, 4), ("ring8", 8, 320, 240, 1, 2)])
def test_seed_run_matches_oracle(gpu_available, name, views, w, h, level, csize):
    import pmvs_amd as P
    inp, p = P.synth_scene(views, w, h, level=level, csize=csize, supersample=2)
    g, o, pts, sg, stg, so, sto = run_pair(inp)
    assert len(so) > 0
    same_seeds(sg, so)
    for k in ("trial", "pass", "fail0", "fail1"):
        assert stg[k] == sto[k], k
    assert stg["refined"] >= stg["trial"]
    g.close()
    o.close()


@pytest.mark.parametrize("lookahead,near", [(1, 2048), (1, 1), (4, 16), (64, 100000)])
def test_seed_run_batch_invariance(gpu_available, monkeypatch, lookahead, near):
    """The speculative batches -- their size, how many images ahead they may request candidates of
    (PMVS_SEED_LOOKAHEAD) and how many cells past the replay cursor every walk re-visits
    (PMVS_SEED_NEAR) -- change how many candidates are refined, never the result."""
    import pmvs_amd as P
    inp, p = P.synth_scene(8, 320, 240, level=1, csize=2, supersample=2)
    g = P.Scene(inp)
    pts = features(g, inp)
    monkeypatch.setenv("PMVS_SEED_LOOKAHEAD", "1")
    monkeypatch.setenv("PMVS_SEED_NEAR", "100000000")
    ref, st_ref = g.seed_run(pts, batch=1)
    monkeypatch.setenv("PMVS_SEED_LOOKAHEAD", str(lookahead))
    monkeypatch.setenv("PMVS_SEED_NEAR", str(near))
    for b in (3, 64, 100000):
        got, st = g.seed_run(pts, batch=b)
        same_seeds(got, ref)
        assert st["trial"] == st_ref["trial"]
        if near >= 2048:  # a narrow walk window may need more rounds than batch 1's full walks
            assert st["rounds"] <= st_ref["rounds"]
    g.close()


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_seed_matrix(gpu_available, cfg):
    inp, p = build(CONFIGS[cfg])
    g, o, pts, sg, stg, so, sto = run_pair(inp, batch=512)
    same_seeds(sg, so)
    assert [stg[k] for k in ("trial", "pass", "fail0", "fail1")] == [sto[k] for k in ("trial", "pass", "fail0", "fail1")]
    g.close()
    o.close()


def test_c1_end_to_end(gpu_available):
    """C1 (3 views, 640x480, level 2, csize 4): features -> seeds -> 3 x (expand, filter) on the
    device equals the oracle's seeds and loop at the reference's single-thread schedule."""
    import pmvs_amd as P
    inp, p = P.synth_scene(3, 640, 480, level=2, csize=4, supersample=2)
    g, o, pts, sg, stg, so, sto = run_pair(inp)
    same_seeds(sg, so)
    mg, _ = g.run_loop(sg, inp.threshold, wave=1)
    mo, _ = o.run_loop(so, inp.threshold, wave=1)
    assert len(mg) == len(mo) > len(sg)
    assert mg.tobytes() == mo.tobytes()
    g.close()
    o.close()
