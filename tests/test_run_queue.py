"""CPU test: the expansion queue as sorted runs (cmvs-pmvs_amd/csrc/pmvs_queue.h, the host side of
CExpand's priority queue, expand.hpp:31 / expand.cpp:82-86,251) pops exactly the sequence a single
binary heap over the same keys pops -- random waves of pushes with many equal _tmp values and -0.0,
interleaved with batch pops of random size."""
import ctypes as C
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rq(tmp_path_factory):
    so = tmp_path_factory.mktemp("rq") / "librq.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(ROOT, "cmvs-pmvs_amd", "csrc"),
                    os.path.join(ROOT, "tests", "csrc", "run_queue_test.cpp"), "-o", str(so)], check=True)
    L = C.CDLL(str(so))
    L.run_queue_check.argtypes = [C.c_uint, C.c_int, C.c_int, C.POINTER(C.c_longlong)]
    return L


@pytest.mark.parametrize("seed,nwaves,initial", [(1, 50, 5000), (2, 200, 0), (3, 5, 100000), (4, 300, 20000)])
def test_run_queue_pops_like_one_heap(rq, seed, nwaves, initial):
    n = C.c_longlong()
    rc = rq.run_queue_check(seed, nwaves, initial, C.byref(n))
    assert rc == 0, rc
    assert n.value > initial
