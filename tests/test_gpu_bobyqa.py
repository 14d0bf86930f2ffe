"""Device BOBYQA (reverse-communication state machine, bobyqa_dev.h) vs the CPU oracle's
BOBYQA (oracle/bobyqa_oracle.h) on analytic objectives: identical final x, f, evaluation count
and NLopt result code, bit for bit, in both the lane-per-problem and wave-per-problem layouts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_device_bobyqa_matches_oracle(gpu_available, oracle_mod, mode, kind):
    import pmvs_amd as P
    rng = np.random.default_rng(10 * kind + mode)
    n = 256
    x0 = np.zeros((n, 3))
    x0[:, 1:] = rng.uniform(-20, 20, (n, 2))
    x0[0] = 0
    maxeval = 1000 if kind != 1 else 300   # Rosenbrock also exercises MAXEVAL termination
    out, ms = P.selftest_bobyqa(kind, x0, mode=mode, maxeval=maxeval)
    for i in range(n):
        rc, xo, fo, rec = oracle_mod.bobyqa_test(kind, x0[i], maxeval=maxeval)
        assert int(out[i, 5]) == rc
        assert int(out[i, 4]) == len(rec)
        assert np.array_equal(out[i, :3].view(np.uint64), xo.view(np.uint64)), i
        assert out[i, 3] == fo
