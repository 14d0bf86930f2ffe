"""BASELINE.json configs[4] (C5) at its full per-GPU size, on one GPU.

C5 -- one CMVS cluster of maximage 70 at 8K (70 views, 7680x4320, level 0), the per-GPU unit of the
1000-view configuration: one full loop iteration (expand + filter) with the model checks, and the
first expansion wave against the oracle record for record.  Its own module, so that no other
test's scenes hold device memory while it runs (the model reaches ~50 M patches of 1608 B).
"""
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


@pytest.mark.timeout(900)
def test_c5_cluster_8k_one_iteration(gpu_available, oracle_mod):
    import bench
    import pmvs_amd as P
    t0 = time.perf_counter()
    lap = lambda what: print(f"[c5 {time.perf_counter() - t0:6.1f} s] {what}", flush=True)  # noqa: E731
    # supersample 1: the host renders 70 views of 33 Mpx in ~25 s instead of ~90 s at 2 (r06k), which keeps
    # the GPU suite inside the driver's step; the scene is the same ring at its full 8K size
    inp, sp = P.synth_scene(70, 7680, 4320, level=0, supersample=1, nthreads=16)
    lap("scene rendered")
    g = P.Scene(inp)
    cands = P.synth_candidates(sp, inp.projections, 5000, seed=0x5EED)
    r, _ = g.refine_batch(cands)
    seeds = P.patches_from_refined(r)
    # the first wave of the iteration-1 expansion (~30 k candidates), device vs oracle, record for record
    ncc, before, depth, cthr = bench.iteration_thresholds(inp.threshold, 0)
    kw = dict(wave=32768, count_threshold=cthr, after_seeds=True, min_candidates=131072)
    g.set_thresholds(ncc, before, depth)
    cap = len(seeds) + 600000
    g_out, g_alive, g_st = g.expand_run(seeds, cap=cap, max_waves=1, **kw)
    lap("device: scene, seeds, first wave")
    o = oracle_mod.OracleScene(inp)
    o.set_thresholds(ncc, before, depth)
    o_out, o_alive, o_st = o.expand_run(seeds, cap=cap, nthreads=_threads(), max_waves=1, **kw)
    o.close()
    lap("oracle first wave")
    print(f"C5 first waves: {o_st}")
    assert o_st["added"] > 10000
    assert all(g_st[k] == o_st[k] for k in o_st), (g_st, o_st)
    assert bench.patch_mismatches(g_out, o_out) == 0 and np.array_equal(g_alive, o_alive)
    del g_out, o_out
    # one full loop iteration on the device (the C5 per-GPU unit)
    g.set_thresholds(*bench.iteration_thresholds(inp.threshold, 0)[:2], 0)
    model, log = g.run_loop(seeds, inp.threshold, iterations=1, wave=32768, min_candidates=131072)
    g.close()
    lap("device iteration + model fetch")
    checks = bench.model_checks(model, inp, ["x"])
    lap("model checks")
    print(f"C5 one iteration: {log[0]['expand']['added']} added, {len(model)} kept, "
          f"{log[0]['expand']['wall_ms'] / 1e3:.1f} s expand, {log[0]['filter']['kernel_ms'] / 1e3:.1f} s filter; {checks}")
    assert checks["ok"] and checks["sphere_residual_p99"] < 0.01, checks
    assert log[0]["expand"]["added"] > 10_000_000
