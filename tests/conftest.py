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
    _Heartbeat.start()


class _Heartbeat:
    """A line every 50 s while one test runs longer than that (the full-size parity tests run for
    minutes): on the session's own stderr, which pytest's capture does not redirect, and appended to
    gpurun_out/heartbeat.txt on the GPU box -- a command that prints nothing for minutes is taken
    for a hung one there."""
    current = None
    since = 0.0

    @classmethod
    def start(cls):
        import threading
        import time
        try:
            fd = os.dup(2)
        except OSError:
            return
        out = None
        root = os.environ.get("GRAFT_REPO_ROOT")
        if root:
            os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
            out = os.path.join(root, "gpurun_out", "heartbeat.txt")

        def run():
            while True:
                time.sleep(50)
                cur, t0 = cls.current, cls.since
                if cur is None or time.time() - t0 < 45:
                    continue
                line = f"[heartbeat] {cur}: {time.time() - t0:.0f} s\n"
                try:
                    os.write(fd, line.encode())
                    if out:
                        with open(out, "a") as f:
                            f.write(line)
                except OSError:
                    pass

        threading.Thread(target=run, daemon=True).start()


def pytest_runtest_logstart(nodeid, location):
    import time
    _Heartbeat.current, _Heartbeat.since = nodeid, time.time()


def pytest_runtest_logfinish(nodeid, location):
    _Heartbeat.current = None


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _make(path):
    """Build in-tree, unless the built artefacts are already newer than every source (the GPU box
    receives the prebuilt libraries without the object files: rebuilding there is not needed)."""
    if os.path.basename(path) == "cmvs-pmvs_amd":
        # each artefact against its own inputs: make only rebuilds what is stale, but the object
        # files do not travel, so any make call on the box would recompile the whole library
        csrc = os.path.join(path, "csrc")
        inc = [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
        mk = [os.path.join(path, "Makefile")]
        lib_srcs = [os.path.join(csrc, f) for f in os.listdir(csrc) if f not in ("pmvs2_main.cpp", "genoption_main.cpp")]
        deps = {"libpmvs_amd.so": lib_srcs + inc + mk,
                "pmvs2": [os.path.join(csrc, "pmvs2_main.cpp")] + inc,
                "genOption": [os.path.join(csrc, "genoption_main.cpp")]}
        if all(os.path.exists(os.path.join(path, o)) and os.path.getmtime(os.path.join(path, o)) >= _newest(d)
               for o, d in deps.items()):
            return
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
