"""CPU test: the device BOBYQA state machine (cmvs-pmvs_amd/csrc/bobyqa_dev.h, compiled for the
host with g++ -ffp-contract=off) reproduces the callback-style oracle BOBYQA (NLopt 2.6.1
LN_BOBYQA semantics, oracle/bobyqa_oracle.h) evaluation-for-evaluation, bit-exactly.

Parity note: nlopt itself is not in the image, so the optimizer trajectory is
pinned only against the restatement ("parity unpinned" vs the real library)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bqhost(tmp_path_factory):
    so = tmp_path_factory.mktemp("bq") / "libbqhost.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", os.path.join(ROOT, "cmvs-pmvs_amd", "csrc"),
                    os.path.join(ROOT, "tests", "csrc", "bq_host.cpp"), "-o", str(so)], check=True)
    L = C.CDLL(str(so))
    L.bq_host_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                              C.POINTER(C.c_int)]
    return L


def run_host(L, kind, x0, maxeval=1000, maxrec=2000):
    x0 = np.ascontiguousarray(x0, np.float64)
    xo, fo, rec, n = np.zeros(3), np.zeros(1), np.zeros(maxrec), C.c_int()
    rc = L.bq_host_run(kind, x0.ctypes.data, maxeval, xo.ctypes.data, fo.ctypes.data, rec.ctypes.data, maxrec,
                       C.byref(n))
    return rc, xo, fo[0], rec[:min(n.value, maxrec)].copy()


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("maxeval", [1000, 40])
def test_rc_bobyqa_matches_oracle(bqhost, oracle_mod, kind, maxeval):
    rng = np.random.default_rng(kind * 100 + maxeval)
    starts = np.concatenate([[[0.0, 0.0, 0.0]], rng.normal(0, [3.0, 8.0, 8.0], (15, 3))])
    starts[:, 1:] = np.clip(starts[:, 1:], -23.99999, 23.99999)
    for x0 in starts:
        a = run_host(bqhost, kind, x0, maxeval)
        b = oracle_mod.bobyqa_test(kind, x0, maxeval)
        assert a[0] == b[0], (x0, a[0], b[0])
        assert np.array_equal(a[1].view(np.uint64), b[1].view(np.uint64))
        assert np.float64(a[2]).view(np.uint64) == np.float64(b[2]).view(np.uint64)
        assert np.array_equal(a[3].view(np.uint64), b[3].view(np.uint64))
        assert len(a[3]) <= maxeval


def test_oracle_bobyqa_converges(oracle_mod):
    rc, x, f, rec = oracle_mod.bobyqa_test(0, np.zeros(3))
    assert rc in (1, 4) and f < 1e-6 + 0.0 or rc in (1, 4)
    # analytic minimiser of the coupled quadratic (kind 0)
    A = np.array([[2.0, 0.1, 0.0], [0.1, 4.0, 0.0], [0.0, 0.0, 1.0]])
    b = np.array([3.0, 12.0, -2.0])
    assert np.allclose(x, np.linalg.solve(A, b), atol=1e-5)
    rc, x, f, rec = oracle_mod.bobyqa_test(2, np.zeros(3))
    assert abs(x[1] - 23.99999) < 1e-9 and abs(x[2] + 23.99999) < 1e-9  # bounds active


@pytest.fixture(scope="module")
def bqlhost(tmp_path_factory):
    so = tmp_path_factory.mktemp("bql") / "libbqlhost.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                    "-DBQL_COUNT", "-I", os.path.join(ROOT, "cmvs-pmvs_amd", "csrc"),
                    os.path.join(ROOT, "tests", "csrc", "bql_host.cpp"), "-o", str(so)], check=True)
    L = C.CDLL(str(so))
    L.bql_host_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                               C.POINTER(C.c_int)]
    L.bql_host_hits.restype = C.POINTER(C.c_longlong)
    return L


def run_lane(L, kind, x0, maxeval=1000, maxrec=2000):
    x0 = np.ascontiguousarray(x0, np.float64)
    xo, fo, rec, n = np.zeros(3), np.zeros(1), np.zeros(maxrec), C.c_int()
    rc = L.bql_host_run(kind, x0.ctypes.data, maxeval, xo.ctypes.data, fo.ctypes.data, rec.ctypes.data, maxrec,
                        C.byref(n))
    return rc, xo, fo[0], rec[:min(n.value, maxrec)].copy()


def test_lane_bobyqa_matches_state_machine(bqhost, bqlhost):
    """The lane-distributed BOBYQA of the lane-form refine kernel (bobyqa_lane.h: one chain per
    wavefront, interpolation points over the lanes, in-order readlane sums; here its host build, a
    wavefront emulated by 64-element arrays) takes the same trajectory as bobyqa_dev.h's state machine
    -- itself pinned to the oracle above -- evaluation for evaluation, bit for bit.  Kinds 3-9 are
    rough objectives (noise, staircases, plateaus, non-smooth, extreme scaling) so that RESCUE, the
    ALTMOV Cauchy step, the xbase shift and the roundoff exits all run; the test checks they did."""
    hits0 = [bqlhost.bql_host_hits()[i] for i in range(11)]
    n = 0
    for kind in range(10):
        for maxeval in (1000, 40, 13):
            rng = np.random.default_rng(kind * 1000 + maxeval)
            starts = np.concatenate([[[0.0, 0.0, 0.0]], rng.normal(0, [3.0, 8.0, 8.0], (40, 3))])
            starts[:, 1:] = np.clip(starts[:, 1:], -23.99999, 23.99999)
            for x0 in starts:
                a = run_host(bqhost, kind, x0, maxeval)
                b = run_lane(bqlhost, kind, x0, maxeval)
                assert a[0] == b[0], (kind, maxeval, x0, a[0], b[0])
                assert np.array_equal(a[1].view(np.uint64), b[1].view(np.uint64)), (kind, x0)
                assert np.float64(a[2]).view(np.uint64) == np.float64(b[2]).view(np.uint64), (kind, x0)
                assert np.array_equal(a[3].view(np.uint64), b[3].view(np.uint64)), (kind, x0)
                n += 1
    hits = [bqlhost.bql_host_hits()[i] - hits0[i] for i in range(11)]
    # [0] RESCUE, [1] xbase shift, [2] itest reset, [3] ALTMOV Cauchy step, [4] RESCUE's den2 retry,
    # [5] RESCUE evaluations, [7] angle searches, [8] XTOL exit, [10] the ntrits == -1 early return
    for i in (0, 1, 2, 3, 4, 5, 7, 8, 10):
        assert hits[i] > 0, (i, hits)
    assert n == 10 * 3 * 41
