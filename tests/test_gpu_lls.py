"""GPU parity of the device least squares (lls5_wave, Cmylapack::lls with Eigen JacobiSVD
semantics) against the oracle's restatement, bit for bit, on random, quadric-fit-shaped,
rank-deficient and degenerate systems."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def systems():
    rng = np.random.default_rng(11)
    out = []
    for n in (6, 7, 9, 20, 64, 65, 200, 1024):
        for _ in range(6):
            fx, fy = rng.normal(0, 1, n).astype(np.float32), rng.normal(0, 1, n).astype(np.float32)
            A = np.stack([fx * fx, fy * fy, fx * fy, fx, fy], 1).astype(np.float32)
            out.append((A, (0.2 * fx * fx - fy + rng.normal(0, 0.05, n)).astype(np.float32)))
    fx = rng.normal(0, 1, 12).astype(np.float32)
    out.append((np.stack([fx * fx, 0 * fx, 0 * fx, fx, 0 * fx], 1).astype(np.float32), fx.copy()))  # collinear
    out.append((np.tile(np.float32([[0.25, 0.0625, 0.125, 0.5, 0.25]]), (8, 1)), np.full(8, 0.7, np.float32)))
    out.append((np.zeros((7, 5), np.float32), np.ones(7, np.float32)))
    out.append((rng.normal(0, 1e-20, (10, 5)).astype(np.float32), rng.normal(0, 1, 10).astype(np.float32)))
    return out


def test_lls_matches_oracle(gpu_available, oracle_mod):
    import pmvs_amd as P
    sy = systems()
    got = P.selftest_lls(sy)
    for k, (A, b) in enumerate(sy):
        want = oracle_mod.lls5(A, b)
        assert got[k].tobytes() == want.tobytes(), (k, got[k], want)
