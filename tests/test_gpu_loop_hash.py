"""pmvs_loop_hash: the device digest of a loop result that stays in HBM (bench.py checks with it that
every timed repetition gives the same model without fetching it).  The digest must equal the same
function evaluated in numpy on the fetched records, and change when one record changes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = np.uint64(0x9E3779B97F4A7C15)


def mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def digest(model):
    """model_digest_kernel's function: sum over records r and words w of
    mix64(word ^ (w << 32) ^ r * golden), xor the record count."""
    n = len(model)
    words = np.ascontiguousarray(model).view(np.uint32).reshape(n, -1).astype(np.uint64)
    w = (np.arange(words.shape[1], dtype=np.uint64) << np.uint64(32))[None, :]
    r = (np.arange(n, dtype=np.uint64) * GOLD)[:, None]
    with np.errstate(over="ignore"):
        h = mix64(words ^ w ^ r).sum(dtype=np.uint64)
    return int(h ^ np.uint64(n))


def test_loop_hash_matches_fetched_model(gpu_available):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    try:
        cands = P.synth_candidates(p, inp.projections, 300, seed=3)
        r, _ = g.refine_batch(cands)
        seeds = P.patches_from_refined(r)
        n, log = g.run_loop(seeds, inp.threshold, iterations=2, wave=256, fetch=False)
        assert n == log[-1]["patches"] > 1000
        h = g.loop_hash()
        assert g.loop_hash() == h  # does not consume the result
        model = g.loop_fetch(n)
        assert digest(model) == h
        ref, _ = g.run_loop(seeds, inp.threshold, iterations=2, wave=256)  # the fetching path: same model
        assert ref.tobytes() == model.tobytes()
        changed = model.copy()
        changed["ncc"][n // 2] = np.nextafter(changed["ncc"][n // 2], np.float32(2))
        assert digest(changed) != h
    finally:
        g.close()
