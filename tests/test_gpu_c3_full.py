"""The headline configuration at full size (BASELINE.json configs[2], C3: 50 views 3840x2160,
level 0) -- the bench's own scene and seeds (bench.py: synth_scene(..., seed 0x504D5653), 5000
seed candidates with rank_seed(0)):

1. One loop step on the device, its model checked by the bench's size-independent invariants, and
   the first expansion waves of every loop iteration compared record for record with the CPU
   oracle (bench.py loop_samples -> parity_c3_first_waves; bench.py exits 3 on a mismatch).
2. One whole CFilter::run pass at 4K (filter.cpp:13-27: filterOutside, filterExact, filterNeighbor,
   filterSmallGroups over 104 M cells): the device's iteration-1 model (the full first expansion,
   about 4.2 M patches) filtered on the device and by the oracle's filter_run -- keep flags, counts
   and the updated records (images, grids, vimages, vgrids, flags) compared record for record.
"""
import argparse
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def c3(gpu_available):
    import bench
    import pmvs_amd as P
    inp, sp = P.synth_scene(50, 3840, 2160, level=0, supersample=2, nthreads=16, seed=0x504D5653)
    scene = P.Scene(inp)
    cands = P.synth_candidates(sp, inp.projections, 5000, seed=bench.rank_seed(0))
    res, _ = scene.refine_batch(cands)
    seeds = P.patches_from_refined(res)
    yield bench, P, inp, scene, seeds
    scene.close()


@pytest.mark.timeout(900)
def test_c3_full_size_step_and_first_waves_match_oracle(c3):
    bench, P, inp, scene, seeds = c3
    model, log = scene.run_loop(seeds, inp.threshold, iterations=3, wave=32768, min_candidates=131072)
    checks = bench.model_checks(model, inp, ["x"])
    print(f"C3 step: {[it['patches'] for it in log]} patches, {sum(it['expand']['added'] for it in log)} added; {checks}")
    assert checks["ok"] and checks["sphere_residual_p99"] < 0.01, checks
    assert log[0]["expand"]["added"] > 3_000_000
    del model
    # iteration 1 here (every bench.py run samples all three iterations: parity_c3_first_waves)
    args = argparse.Namespace(iterations=3, cpu_iterations=1, cpu_waves=2, cpu_waves_late=0, cpu_seconds=1.0,
                              cpu_threads=0, cpu_filter_every=0, wave=32768, min_candidates=131072)
    _, parity = bench.loop_samples(P, scene, inp, seeds, args, [it["expand"]["added"] for it in log])
    print(f"first waves: {parity}")
    assert all(p["ok"] for p in parity), parity
    assert parity[0]["added"] > 10000 and parity[0]["mismatched_records"] == 0


@pytest.mark.timeout(900)
def test_c3_4k_filter_pass_matches_oracle(c3, oracle_mod):
    bench, P, inp, scene, seeds = c3
    ncc, before, depth, cthr = bench.iteration_thresholds(inp.threshold, 0)
    scene.set_thresholds(ncc, before, depth)
    model, _, st = scene.expand_run(seeds, wave=32768, count_threshold=cthr, after_seeds=True, min_candidates=131072,
                                    cap=len(seeds) + (8 << 20))
    print(f"iteration-1 model: {len(model)} patches ({st['added']} added in {st['waves']} waves)")
    assert len(model) > 3_000_000
    g_out, g_keep, g_st = scene.filter_run(model)
    o = oracle_mod.OracleScene(inp)
    o.set_thresholds(ncc, before, depth)
    oracle_mod.lib().oracle_set_threads(bench.host_cpus()["usable"])
    import time
    t0 = time.perf_counter()
    o_out, o_keep, o_counts = o.filter_run(model)
    t_o = time.perf_counter() - t0
    o.close()
    counts = [g_st[k] for k in ("removed_outside", "removed_exact", "removed_neighbor", "removed_groups")]
    print(f"4K filter pass: device {counts} in {g_st['kernel_ms']:.0f} ms, oracle {o_counts.tolist()} in {t_o:.1f} s")
    assert counts == o_counts.tolist()
    assert sum(counts) > 1000  # the pass removes patches: the comparison is not vacuous
    assert np.array_equal(g_keep, o_keep)
    assert bench.patch_mismatches(g_out, o_out) == 0
