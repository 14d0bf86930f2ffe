"""CPU tests of the oracle's Cmylapack::lls restatement (mylapack.cpp:102-149: Eigen
JacobiSVD(ComputeThinU | ComputeThinV).solve in double, cast to float), used by filterQuad:
full-rank systems give the least-squares solution, rank-deficient ones (collinear or coincident
neighbours) the minimum-norm solution with Eigen's rank threshold (5 eps s_max) -- the property a
plain QR solve lacks.  numpy's SVD lstsq is the independent check (parity with Eigen itself is
unpinned: Eigen is absent from the image)."""
import numpy as np
import pytest


def quad_rows(fx, fy):
    return np.stack([fx * fx, fy * fy, fx * fy, fx, fy], 1).astype(np.float32)


@pytest.mark.parametrize("n", [6, 7, 20, 150])
def test_full_rank_matches_lstsq(oracle_mod, n):
    rng = np.random.default_rng(n)
    for _ in range(20):
        fx, fy = rng.normal(0, 1, n), rng.normal(0, 1, n)
        A = quad_rows(fx, fy)
        b = (0.3 * fx * fx - 0.2 * fy + rng.normal(0, 0.01, n)).astype(np.float32)
        x = oracle_mod.lls5(A, b)
        ref = np.linalg.lstsq(A.astype(np.float64), b.astype(np.float64), rcond=None)[0]
        assert np.allclose(x, ref, rtol=1e-5, atol=1e-6)


def test_rank_deficient_min_norm(oracle_mod):
    """Neighbours on a line (fy = 0): columns fy^2, fx*fy, fy vanish -> rank 2; coincident points
    -> rank 1.  The solution is the minimum-norm one, finite, with zeros on the null columns."""
    rng = np.random.default_rng(3)
    fx = rng.normal(0, 1, 12)
    A = quad_rows(fx, np.zeros(12))
    b = (0.5 * fx * fx + 0.1 * fx).astype(np.float32)
    x = oracle_mod.lls5(A, b)
    ref = np.linalg.lstsq(A.astype(np.float64), b.astype(np.float64), rcond=None)[0]
    assert np.all(np.isfinite(x))
    assert np.allclose(x, ref, rtol=1e-5, atol=1e-6)
    assert x[1] == 0 and x[2] == 0 and x[4] == 0
    A1 = np.tile(np.array([[0.25, 0.0625, 0.125, 0.5, 0.25]], np.float32), (8, 1))
    b1 = np.full(8, 0.7, np.float32)
    x1 = oracle_mod.lls5(A1, b1)
    ref1 = np.linalg.lstsq(A1.astype(np.float64), b1.astype(np.float64), rcond=None)[0]
    assert np.allclose(x1, ref1, rtol=1e-5, atol=1e-7)


def test_zero_system(oracle_mod):
    x = oracle_mod.lls5(np.zeros((7, 5), np.float32), np.ones(7, np.float32))
    assert np.all(x == 0)
