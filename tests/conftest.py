"""Shared test fixtures.  `-m gpu` tests need a HIP device; everything else runs on the CPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def _make(path):
    subprocess.run(["make", "-C", path, "-s"], check=True)


@pytest.fixture(scope="session")
def product_lib():
    _make(os.path.join(ROOT, "cmvs-pmvs_amd"))
    import pmvs_amd
    return pmvs_amd.load_library()


@pytest.fixture(scope="session")
def oracle_mod():
    _make(os.path.join(ROOT, "oracle"))
    import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def gpu_available(product_lib):
    import pmvs_amd
    if pmvs_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X (no CPU fallback)")
    return True


def small_scene(num_views=6, width=320, height=240, level=1, num_targets=None, **kw):
    import pmvs_amd
    inp, p = pmvs_amd.synth_scene(num_views, width, height, level=level, num_targets=num_targets,
                                  supersample=2, **kw)
    return inp, p
