"""Uninitialised-memory hunt (pmvs_api.cpp / pmvs_filter.hip poison_alloc): with
PMVS_POISON_ALLOC=<byte> every new device allocation of the scene is filled with that byte, so a
kernel that reads memory no kernel wrote changes the result.  The loop (expand -> refine -> filter,
pmvs_run_loop) and a refine batch must give byte-identical output with two different poison bytes
and without poisoning.  The variable is read once per process, so each run is a child process."""
import hashlib
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, sys
sys.path.insert(0, sys.argv[1])
import pmvs_amd as P
inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2, hard=True)
g = P.Scene(inp)
cands = P.synth_candidates(p, inp.projections, 400, seed=9)
r, _ = g.refine_batch(cands)
seeds = P.patches_from_refined(r)
out, log = g.run_loop(seeds, inp.threshold, wave=256, min_candidates=512)
g.close()
print(hashlib.sha1(r.tobytes()).hexdigest(), hashlib.sha1(out.tobytes()).hexdigest(), len(out))
"""


def _run(poison):
    env = dict(os.environ)
    env.pop("PMVS_POISON_ALLOC", None)
    if poison is not None:
        env["PMVS_POISON_ALLOC"] = str(poison)
    res = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "cmvs-pmvs_amd")], env=env,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    return res.stdout.split()


@pytest.mark.timeout(600)
def test_poisoned_allocations_do_not_change_results(gpu_available):
    base = _run(None)
    assert int(base[2]) > 1000
    for byte in (0xAB, 0x00):
        assert _run(byte) == base, f"poison byte {byte:#x} changed the result"
