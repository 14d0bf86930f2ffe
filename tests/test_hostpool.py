"""CPU test: the persistent host thread pool of the refine's start-angle step
(cmvs-pmvs_amd/csrc/pmvs_hostpool.h): exact coverage of the range for any thread count, concurrent
callers (a busy pool is declined, the caller runs alone), and a forked child that declines instead
of waiting for workers it does not have."""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hostpool(tmp_path):
    so = tmp_path / "libhp.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-I",
                    os.path.join(ROOT, "cmvs-pmvs_amd", "csrc"), os.path.join(ROOT, "tests", "csrc", "hostpool_test.cpp"),
                    "-o", str(so)], check=True)
    assert C.CDLL(str(so)).hostpool_check() == 0
