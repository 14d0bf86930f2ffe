"""CPU checks of the expansion oracle (oracle/expand_oracle.h, a restatement of
PMVS3::CExpand::run, expand.cpp:17-406).  Parity unpinned against the reference binary (its
expansion needs the whole findMatch runtime, unbuildable here): these are the invariants the
reference's own bookkeeping implies, on a synthetic ring."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def seeds(oracle_mod):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    o = oracle_mod.OracleScene(inp)
    c = P.synth_candidates(p, inp.projections, 300, seed=3)
    r = o.refine_batch(c, nthreads=8)
    pa = P.patches_from_refined(r[0] if isinstance(r, tuple) else r)
    yield P, inp, o, pa
    o.close()


@pytest.mark.parametrize("depth,wave", [(1, 1), (1, 64), (2, 1)])
def test_expand_invariants(seeds, depth, wave):
    P, inp, o, pa = seeds
    o.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
    out, alive, st = o.expand_run(pa, wave=wave, cap=100000)
    n0 = len(pa)
    assert st["added"] == len(out) - n0 and st["added"] > 5 * n0
    assert st["candidates"] == st["fail_prep"] + st["fail_pre"] + st["fail_post"] + st["fail_commit"] + st["added"]
    if wave == 1:
        assert st["fail_commit"] == 0 and st["waves"] == st["parents"]
    new = out[n0:]
    assert (alive == 1).all()
    assert (new["ncc"] >= inp.threshold).all()  # postProcess acceptance (optim.cpp:2036)
    assert (new["flag"] == 1).all() and (new["fix"] == 0).all()
    assert (new["num_images"] >= 2).all()
    for q in new[:200]:
        imgs = q["images"][:q["num_images"]]
        assert len(set(imgs.tolist())) == len(imgs) and (imgs >= 0).all() and (imgs < len(inp.images)).all()
        vims = set(q["vimages"][:q["num_vimages"]].tolist())
        assert not (vims & set(imgs.tolist()))  # setVImagesVGrids skips used images
    # every parent that failed a direction recorded it in _dflag (expand.cpp:99-101)
    failed = st["candidates"] - st["added"]
    bits = sum(bin(int(x)).count("1") for x in out["dflag"])
    assert bits == failed


def test_expand_deterministic_and_empty(seeds):
    P, inp, o, pa = seeds
    o.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    a = o.expand_run(pa[:80], wave=16, cap=100000)
    b = o.expand_run(pa[:80], wave=16, cap=100000)
    assert np.array_equal(a[0].view(np.uint8), b[0].view(np.uint8)) and a[2] == b[2]
    out, alive, st = o.expand_run(pa[:0], wave=16, cap=16)
    assert len(out) == 0 and st["parents"] == 0


def test_loop_oracle(seeds):
    """Three (expand, filter, updateThreshold) iterations from seeds grow then thin the model."""
    P, inp, o, pa = seeds
    model, log = o.run_loop(pa, inp.threshold, iterations=3, wave=256)
    assert [x["depth"] for x in log] == [1, 2, 3]
    assert log[0]["expand"]["added"] > 5 * len(pa)
    assert len(model) == log[-1]["patches"] > len(pa)
    assert all(x["expand"]["parents"] > 0 for x in log)


def test_candidate_centres_match_reference(oracle_mod):
    """findEmptyBlocks' candidate centres (expand.cpp:176-177: float angle, double cos/sin,
    Vec4f scaling) from the oracle == the same two reference lines evaluated with the
    reference's own headers in oracle/_ref (tests/golden/expand_dirs.npz), bit for bit.  The
    earlier double-angle restatement differed on ~22 % of these centres."""
    import os
    import numpy as np
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "expand_dirs.npz")))
    out = np.zeros_like(g["ref_coords"])
    oracle_mod.lib().oracle_expand_dirs(g["coord"].ctypes.data, g["normal"].ctypes.data, g["radius"].ctypes.data,
                                        len(g["coord"]), out.ctypes.data)
    assert out.view(np.uint32).tobytes() == g["ref_coords"].view(np.uint32).tobytes()
