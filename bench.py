#!/usr/bin/env python3
"""bench.py -- MI355X PMVS2 dense-matching throughput (BASELINE.json metric), one JSON line on rank 0.

Workload (default, BASELINE.json configs[2] "C3" -- the metric's "50-view 4K synthetic"): a
synthetic 50-view 3840x2160 textured-sphere ring, level 0, csize 2, wsize 7, minImageNum 3,
threshold 0.7.  Setup (untimed): render the views, build the scene on the device, and make the
seed model: --seed-mode features runs the seed phase on the device (Harris/DoG features +
CSeed::run); --seed-mode synthetic (default) refines --seeds synthetic
seed-path candidates instead.  One step = CFindMatch::run after the seeds: 3 x (CExpand::run -> COptim refine ->
CFilter::run, updateThreshold) through pmvs_run_loop, with the model resident in HBM.

value = refined patches/s: patches the expansion refined and committed to the model
(preProcess -> refinePatch -> postProcess passed, expand.cpp:238) over all ranks / step time.
Also: NCC evals/s (my_f + computeINCC evaluations), refined candidates/s.
roofline: the loop's dominant kernel, refine_split_kernel (the refine batches of >= 10000 candidates):
algorithmic bytes = 588 B x valid textures per my_f evaluation over its HIP-event
time, against 8 TB/s HBM; the smaller batches' lane-form kernel (below 7000 candidates) in roofline.small_batches.
refine_c2: the refine kernel alone on configs[1] (8-view 1920x1080, level 1, 100k candidates).
cpu_baseline: the same metric on the host CPU -- the oracle (CPU restatement) runs the expansions
of the same rank-0 C3 scene from the same models with the same wave schedule (findEmptyBlocks,
preparation and the refinements of a wave on a std::thread pool over every CPU this process may
use, commit serial as in the product): the first --cpu-waves waves of iteration 1 and the whole
expansions of iterations 2 and 3, and a sampled CFilter::run pass per iteration (--cpu-filter-every);
value = the GPU step's patches over the CPU time the per-iteration rates extrapolate for them.  A refine-only rate over synthetic seed candidates is
reported beside it (refine_only).
checks: size-independent properties of the C3 model (identical model from every repetition,
finite geometry, unit normals, image-list invariants, the synthetic sphere's surface residual).

Multi-GPU (`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`), one
process per GPU:
  --mode shard (default for N > 1, strong scaling): all ranks run ONE 50-view scene, the metric's
    "50-view 4K ring at 1/2/4/8 GPUs by target-image sharding" (BASELINE.md); every expansion
    wave's refinements and findEmptyBlocks are split over the ranks, the filter's per-target stages
    run on the target's owner, and the records are all-gathered over RCCL
    (pmvs_scene_set_shard_rccl: a C++ RCCL communicator, device-to-device records).  The model is
    bit-identical to one GPU's.
  --mode cluster (opt-in, weak scaling): each rank owns one CMVS-style cluster -- its own
    50-view scene (rank-seeded texture) -- and runs the loop on it independently, as the
    reference runs one pmvs2 per cluster option file (genOption.cpp:73-108); no data-path
    collective, only barriers and the SUM / MAX reductions of the counters and the time.
  --mode c4 (BASELINE.json configs[3] at 8 GPUs): one ring of --c4-views-per-cluster x N views split
    into N CMVS-style clusters (consecutive targets, each sharing --c4-overlap views with each
    neighbour, as CMVS's ske.dat clusters overlap), one per GPU; the loop exchanges the clusters'
    boundary patches over the native RCCL communicator after every iteration
    (pmvs_scene_set_cluster_rccl).  value = patches all clusters committed / max time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cmvs-pmvs_amd"))

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
BYTES_PER_TEXTURE = 49 * 4 * 3  # wsize^2 samples x 4 texels x 3 B


def refine_kernel_name(cfg):
    """The refine kernel a PMVS_REFINE_CONFIG value launches (pmvs_kernels.hip launch_refine_ws)."""
    if cfg >= 300000:  # lane form: 300000 + lanes per texture (0: from tau; 8 at C3's tau 6)
        return f"refine_lane_kernel<7,{cfg % 100 or 8}>"
    if cfg >= 200000:  # split form: 200000 + LP * 10000 + optimizer wavefronts * 1000 + chains per wavefront
        return f"refine_split_kernel<7,{(cfg // 1000) % 10},{cfg % 1000},{max(1, (cfg // 10000) % 10)}>"
    if cfg >= 100000:  # workgroup form: 100000 + chains * 1000 + optimizer wavefronts * 10 + workgroups per CU
        return f"refine_wg_kernel<7,{(cfg // 1000) % 100},...,{(cfg // 10) % 10}>"
    return f"refine_v2_kernel<7,{cfg // 100},{cfg % 100}>"  # texture slots * 100 + chains per wavefront


# the refine layouts of the batches >= 10000 candidates and below (pmvs_api.cpp Scene::refine_cfg)
_RCFG = int(os.environ.get("PMVS_REFINE_LARGE_CONFIG", os.environ.get("PMVS_REFINE_CONFIG", "226014")))
REFINE_KERNEL = refine_kernel_name(_RCFG)
SMALL_KERNEL = refine_kernel_name(int(os.environ.get("PMVS_REFINE_SMALL_CONFIG", os.environ.get("PMVS_REFINE_CONFIG",
                                                                                                   "300000"))))


_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=("cluster", "shard", "c4"), default=None,
                    help="multi-GPU mode; default shard (ONE 50-view ring over all GPUs, the metric's "
                         "target-image sharding, BASELINE.md); cluster = independent replicas")
    ap.add_argument("--c4-views-per-cluster", type=int, default=25)
    ap.add_argument("--c4-overlap", type=int, default=2)
    ap.add_argument("--views", type=int, default=50)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--level", type=int, default=0)
    ap.add_argument("--seed-mode", choices=("features", "synthetic"), default="synthetic",
                    help="features: the seed phase on the device (Harris/DoG + CSeed::run, findMatch.cpp:187-193); "
                         "synthetic: refine --seeds synthetic seed-path candidates")
    ap.add_argument("--seeds", type=int, default=5000, help="synthetic seed candidates (--seed-mode synthetic)")
    ap.add_argument("--wave", type=int, default=32768)
    ap.add_argument("--min-candidates", type=int, default=131072)
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--c2-candidates", type=int, default=100000)
    ap.add_argument("--no-c2", action="store_true", help="skip the configs[1] refine-kernel side measurement")
    ap.add_argument("--only-c2", action="store_true", help="only the configs[1] refine-kernel measurement (profiling)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="refine-only CPU sample time budget")
    ap.add_argument("--cpu-waves", type=int, default=12,
                    help="expansion waves of loop iteration 1 in the CPU loop sample (iteration 1 holds ~99%% of a "
                         "C3 step's patches; its rate is extrapolated from these waves)")
    ap.add_argument("--cpu-waves-late", type=int, default=0,
                    help="expansion waves of loop iterations 2.. in the CPU loop sample (0 = the whole expansion)")
    ap.add_argument("--cpu-filter-every", type=int, default=8,
                    help="CPU baseline filter sample: the patches whose reference image index is a multiple of this "
                         "(0 = no filter timing)")
    ap.add_argument("--cpu-iterations", type=int, default=3,
                    help="loop iterations sampled by the CPU baseline / full-size parity check (1..iterations)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def pmc_traffic(workload):
    """HBM bytes per refine-kernel launch from the newest committed rocprofv3 PMC summary of the
    same workload (tools/gpu_round.sh + tools/summarize_profiles.py: FETCH_SIZE x2 per
    MI355X_MICROARCH.md + WRITE_SIZE, separate --pmc passes); otherwise null."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        d = json.load(open(f))
        if d.get("workload") != workload:
            continue
        for k, v in d.get("kernels", {}).items():
            base = REFINE_KERNEL.split("<")[0]
            if k.startswith("pmvsdev::" + base) or k.startswith(base):
                return int(v["hbm_bytes_per_launch"]), int(v.get("launches", 0)), os.path.relpath(f, ROOT)
    return None, None, None


def host_cpus():
    """CPUs this process may use: the affinity mask, further limited by a cgroup v2 CPU quota
    (cpu.max) when one is set; with the machine's logical CPU count and model for the record."""
    import math
    logical = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = logical
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, math.ceil(quota)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "logical": logical, "affinity": affinity, "cgroup_quota_cpus": quota, "model": model}


PATCH_SCALARS = ("coord", "normal", "ncc", "dscale", "ascale", "tmp", "timages", "flag", "fix", "num_images",
                 "num_vimages", "dflag")


def patch_mismatches(a, b):
    """Records of two pmvs_patch arrays that differ in any defined field (floats bit for bit, the
    image / vimage lists up to their counts); -1 when the lengths differ."""
    if len(a) != len(b):
        return -1
    bad = np.zeros(len(a), bool)
    for f in PATCH_SCALARS:
        x, y = np.ascontiguousarray(a[f]), np.ascontiguousarray(b[f])
        if x.dtype.kind == "f":
            x, y = x.view(np.uint32), y.view(np.uint32)
        d = x != y
        bad |= d.reshape(len(a), -1).any(axis=1)
    for lst, grd, cnt in (("images", "grids", "num_images"), ("vimages", "vgrids", "num_vimages")):
        k = np.arange(a[lst].shape[1])[None, :]
        m = k < b[cnt][:, None]
        bad |= ((a[lst] != b[lst]) & m).any(axis=1)
        bad |= ((a[grd] != b[grd]).any(axis=2) & m).any(axis=1)
    return int(bad.sum())


def iteration_thresholds(threshold, t):
    """(ncc, before, depth, count_threshold) of loop iteration t (0-based) as pmvs_run_loop / CFindMatch
    set them: before = threshold - 0.3f, both -= 0.05f per iteration, depth 1.., _countThreshold1 4 -> 2
    (findMatch.cpp:23-28, 104) -- float arithmetic."""
    ncc = np.float32(threshold)
    before = np.float32(ncc - np.float32(0.3))
    for _ in range(t):
        ncc = np.float32(ncc - np.float32(0.05))
        before = np.float32(before - np.float32(0.05))
    return float(ncc), float(before), t + 1, 4 if t == 0 else 2


def loop_samples(P, scene, inp, seeds, args, gpu_added):
    """Full-size parity and the loop-level CPU baseline on the rank-0 C3 scene.

    For each sampled loop iteration t the model at the start of t (the seeds, or the device loop's
    model after t iterations) is expanded with the production schedule, once on the device
    (pmvs_expand_run with PMVS_EXPAND_MAX_WAVES) and once by the CPU oracle (the same wave schedule;
    findEmptyBlocks, preparation and refinement on a std::thread pool over every CPU this process may
    use, commit serial): the first --cpu-waves waves of iteration 1 (it holds ~99 % of a C3 step's
    patches) and --cpu-waves-late waves (0: the whole expansion) of iterations 2... parity: the two
    results record for record.  cpu_baseline: each iteration's CPU rate (patches committed per second
    of its waves, the iteration's model setup included) applied to the patches the GPU step commits
    in that iteration (gpu_added[t]): value = sum_t added_t / sum_t (added_t / rate_t)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    cpus = host_cpus()
    threads = args.cpu_threads or cpus["usable"]
    o = O.OracleScene(inp)
    parity, per_iter = [], []
    for t in range(max(1, min(args.cpu_iterations, args.iterations))):
        log(f"parity / CPU sample: iteration {t + 1}")
        if t == 0:
            model = seeds
        else:
            model, _ = scene.run_loop(seeds, inp.threshold, iterations=t, wave=args.wave,
                                      min_candidates=args.min_candidates)
        ncc, before, depth, cthr = iteration_thresholds(inp.threshold, t)
        kw = dict(wave=args.wave, count_threshold=cthr, after_seeds=(t == 0), min_candidates=args.min_candidates)
        waves = args.cpu_waves if t == 0 else args.cpu_waves_late
        if waves > 0:
            cap = len(model) + 16 * args.wave * waves + max(args.min_candidates, 1024) * waves * 6
        else:
            cap = len(model) + max(1 << 20, len(model) // 4)
        scene.set_thresholds(ncc, before, depth)
        g_out, g_alive, g_st = scene.expand_run(model, cap=cap, max_waves=waves, **kw)
        o.set_thresholds(ncc, before, depth)
        o_out, o_alive, o_st = o.expand_run(model, cap=cap, nthreads=threads, max_waves=waves, **kw)
        mism = patch_mismatches(g_out, o_out)
        same_stats = all(g_st[k] == o_st[k] for k in o_st)
        ok = mism == 0 and same_stats and bool(np.array_equal(g_alive, o_alive))
        parity.append({"iteration": t + 1, "model_in": int(len(model)), "waves": int(o_st["waves"]),
                       "whole_expansion": waves <= 0, "candidates": int(o_st["candidates"]),
                       "added": int(o_st["added"]), "records": int(len(o_out)), "mismatched_records": mism,
                       "stats_equal": same_stats, "ok": ok})
        rate = o_st["added"] / max(o.last_wave_s, 1e-9)
        ga = int(gpu_added[t]) if t < len(gpu_added) else 0
        it = {"iteration": t + 1, "waves": int(o_st["waves"]), "whole_expansion": waves <= 0,
              "added": int(o_st["added"]), "wave_s": round(o.last_wave_s, 3), "value": round(rate, 1),
              "gpu_added": ga, "cpu_s_extrapolated": round(ga / max(rate, 1e-9), 2),
              "filter_input": int(len(model)) + ga}
        if waves <= 0 and args.cpu_filter_every > 0:
            # CFilter::run of this iteration on the CPU: the expanded model is exactly the pass's input
            # (the whole expansion ran); a pass over the patches whose reference image index is a
            # multiple of --cpu-filter-every is timed and scaled by the patch count
            alive = o_out[np.asarray(o_alive).astype(bool)]
            sub = alive[(alive["images"][:, 0] % args.cpu_filter_every) == 0]
            O.lib().oracle_set_threads(threads)
            tf = time.perf_counter()
            o.filter_run(sub)
            fs = time.perf_counter() - tf
            it["filter_input"] = int(len(alive))
            it["filter_sample"] = {"patches": int(len(sub)), "s": round(fs, 3)}
            it["filter_s_per_patch"] = fs / max(len(sub), 1)
        per_iter.append(it)
        del g_out, o_out, model
    scene.set_thresholds(*iteration_thresholds(inp.threshold, 0)[:2], 0)
    # refine-only side figure: preProcess -> refinePatch -> postProcess on seed-path candidates
    sp = P.synth_params(len(inp.images), inp.images[0].shape[1], inp.images[0].shape[0], level=inp.level)
    sample = P.synth_candidates(sp, inp.projections, 400000, seed=0xC0FFEE)
    done = acc = 0
    o.set_thresholds(*iteration_thresholds(inp.threshold, 0)[:2], 0)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds and done < len(sample):
        r, rs = o.refine_batch(sample[done:done + 2000], nthreads=threads)
        done += len(r)
        acc += rs["accepted"]
    tr = time.perf_counter() - t0
    o.close()
    # the filter passes: per-patch CPU cost of the sampled passes (mean over iterations for those whose
    # expansion was only sampled, i.e. iteration 1) times each pass's input
    costs = [p["filter_s_per_patch"] for p in per_iter if "filter_s_per_patch" in p]
    for p in per_iter:
        c = p.pop("filter_s_per_patch", None)
        if c is None and costs:
            c = sum(costs) / len(costs)
        p["filter_s_extrapolated"] = round(c * p["filter_input"], 2) if c is not None else None
    tot_added = sum(p["gpu_added"] for p in per_iter)
    tot_s = sum(p["cpu_s_extrapolated"] + (p["filter_s_extrapolated"] or 0.0) for p in per_iter)
    tot_expand_s = sum(p["cpu_s_extrapolated"] for p in per_iter)
    sampled_added = sum(p["added"] for p in per_iter)
    sampled_s = sum(p["wave_s"] for p in per_iter)
    first = per_iter[0]
    cpu = {"value": round(tot_added / max(tot_s, 1e-9), 1), "unit": "refined patches/s", "cores": threads,
           "kind": "port",
           "sample": f"per-iteration CPU rates weighted by the GPU step's own patches (extrapolated): iteration 1 "
                     f"from its first {first['waves']} expansion waves ({first['added']} patches in {first['wave_s']} s), "
                     f"iterations 2..{len(per_iter)} from "
                     + ("their whole expansions" if args.cpu_waves_late <= 0 else f"their first {args.cpu_waves_late} waves")
                     + f" (wave {args.wave}, min_candidates {args.min_candidates}; each iteration starts from the "
                     f"device loop's model, and the same waves run on the device and match record for record, "
                     f"parity_c3_first_waves); plus each iteration's CFilter::run pass: a CPU pass over the "
                     f"patches whose reference image index is a multiple of {args.cpu_filter_every} timed and scaled "
                     f"by the pass's input (iteration 1 at the mean per-patch cost of the later passes); value = "
                     f"sum_t gpu_added_t / sum_t (gpu_added_t / cpu_rate_t + filter_s_t) = {tot_added} patches in "
                     f"{tot_s:.1f} s extrapolated ({tot_expand_s:.1f} s expansion + {tot_s - tot_expand_s:.1f} s "
                     f"filter); oracle/liboracle.so (CPU restatement), {threads} threads",
           "per_iteration": per_iter,
           "expand_only": {"value": round(tot_added / max(tot_expand_s, 1e-9), 1), "unit": "refined patches/s",
                           "sample": "the same, without the filter passes (the round-5 definition)"},
           "sampled": {"value": round(sampled_added / max(sampled_s, 1e-9), 1), "unit": "refined patches/s",
                       "sample": f"the sampled waves pooled, unweighted: {sampled_added} patches in {sampled_s:.2f} s"},
           "host": cpus,
           "refine_only": {"value": round(acc / tr, 1), "unit": "refined patches/s",
                           "sample": f"{done} seed-path candidates, preProcess->refinePatch->postProcess, {tr:.1f} s"}}
    return cpu, parity


def model_checks(model, inp, hashes):
    """Size-independent properties of a C3 loop result (the model is too large for the oracle)."""
    import pmvs_amd as P
    n = len(model)
    coord = model["coord"][:, :3].astype(np.float64)
    normal = model["normal"][:, :3].astype(np.float64)
    ni = model["num_images"]
    tnum = inp.num_targets
    radius = np.linalg.norm(coord, axis=1)  # synthetic scene: the unit sphere
    checks = {
        "model_identical_across_steps": len(set(hashes)) == 1,
        "model_hash": hashes[0] if hashes else None,
        "finite": bool(np.isfinite(model["coord"]).all() and np.isfinite(model["normal"]).all()),
        "unit_normals": bool(np.all(np.abs(np.linalg.norm(normal, axis=1) - 1.0) < 1e-3)),
        "min_images_ok": bool(np.all(ni >= inp.min_image_num)),
        "reference_is_target": bool(np.all(model["images"][:, 0] < tnum)),
        "images_unique": bool(all(len(set(model["images"][i, :ni[i]].tolist())) == ni[i]
                                  for i in range(0, n, max(1, n // 20000)))),
        "sphere_residual_mean": float(np.mean(np.abs(radius - 1.0))),
        "sphere_residual_p99": float(np.percentile(np.abs(radius - 1.0), 99)),
        "ncc_min": float(model["ncc"].min()) if n else None,
    }
    checks["ok"] = all(checks[k] for k in ("model_identical_across_steps", "finite", "unit_normals",
                                           "min_images_ok", "reference_is_target", "images_unique"))
    return checks


def rank_seed(rank: int) -> int:
    return 0x5EED + 7919 * rank


def reduce_over_ranks(dist, counts, elapsed, device):
    """SUM the per-rank counters and MAX the per-rank timed-region length over all ranks.  Works
    with nccl (RCCL) on GPUs and gloo on CPUs."""
    import torch
    totals = torch.tensor([float(c) for c in counts], dtype=torch.float64, device=device)
    tmax = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return totals.tolist(), tmax.item()


def refine_roofline(tex_valid, refine_ms, launches, traffic, traffic_launches, src):
    s = refine_ms / 1e3
    achieved = tex_valid * BYTES_PER_TEXTURE / s / 1e9 if s > 0 else 0.0
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": REFINE_KERNEL,
            "launches": launches, "kernel_ms_avg": round(refine_ms / max(1, launches), 3),
            "algorithmic_bytes_per_launch": int(tex_valid * BYTES_PER_TEXTURE / max(1, launches)),
            "traffic_source": src, "traffic_launches": traffic_launches}


def c2_refine(P, args, dev, rank):
    """configs[1]: the refine kernel alone (preProcess -> refinePatch -> postProcess) on 100k
    seed-path candidates of an 8-view 1920x1080 level-1 ring, candidates resident in HBM."""
    import torch
    inp, sp = P.synth_scene(8, 1920, 1080, level=1, supersample=2, nthreads=16)
    scene = P.Scene(inp, device=dev.index or 0)
    n = args.c2_candidates
    cands = P.synth_candidates(sp, inp.projections, n, seed=rank_seed(rank))
    d_in = torch.from_numpy(cands.view(np.uint8)).to(dev)
    d_out = torch.empty(n * P.REFINED_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    scene.refine_batch_device(d_in.data_ptr(), n, d_out.data_ptr())
    scene.sync()
    stats = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        scene.refine_batch_device(d_in.data_ptr(), n, d_out.data_ptr())
        stats.append(scene.sync())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    scene.close()
    acc = sum(s["accepted"] for s in stats)
    ev = sum(s["evals"] for s in stats)
    tv = sum(s["tex_valid"] for s in stats)
    rms = sum(s["refine_ms"] for s in stats)
    tr, tl, src = pmc_traffic("c2")
    return {"workload": "C2: 8-view 1920x1080 ring, level 1, 100000 seed candidates, refine kernel only",
            "value": round(acc / el, 1), "unit": "refined patches/s", "ncc_evals_per_s": round(ev / el, 1),
            "ms_per_step": round(el / 3 * 1e3, 3),
            "roofline": refine_roofline(tv, rms, 3, tr, tl, src)}


def c4_cluster(P, args, rank, world):
    """Cluster `rank` of a ring of views_per_cluster x world views: target image numbers
    [vpc*rank - ov, vpc*(rank+1) + ov) mod V (every view once at world 1), rendered alone; seeds = the
    synthetic seed candidates of the whole ring whose two images lie in the cluster, refined."""
    vpc, ov = args.c4_views_per_cluster, (args.c4_overlap if world > 1 else 0)
    V = vpc * world
    first = (vpc * rank - ov) % V
    ids = [(first + k) % V for k in range(vpc + 2 * ov)]
    sp = P.synth_params(V, args.width, args.height, level=args.level, supersample=2)
    sp.render_first, sp.render_count = first, len(ids)
    rgb, proj = P.synth_ring(sp, nthreads=16)
    inp = P.SceneInputs(images=[rgb[k] for k in range(len(ids))], projections=proj[ids], num_targets=len(ids),
                        level=args.level)
    return inp, sp, proj, ids


def c4_seeds(P, scene, sp, proj, ids, n):
    cands = P.synth_candidates(sp, proj, n, seed=0x5EED)
    loc = {v: k for k, v in enumerate(ids)}
    keep = [i for i in range(len(cands)) if int(cands["images"][i][0]) in loc and int(cands["images"][i][1]) in loc]
    cs = cands[keep].copy()
    for c in cs:
        c["images"][0] = loc[int(c["images"][0])]
        c["images"][1] = loc[int(c["images"][1])]
    r, _ = scene.refine_batch(cs)
    return P.patches_from_refined(r)


def main():
    args = parse()
    import torch
    import pmvs_amd as P

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    if args.mode is None:
        args.mode = "shard" if world > 1 else "cluster"
    shard = args.mode == "shard" and world > 1
    c4 = args.mode == "c4"
    if args.only_c2:
        c2 = c2_refine(P, args, dev, rank)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "refine_c2": c2}), flush=True)
        return c2

    # ---- scene: one cluster per rank (cluster mode) or one shared scene (shard mode)
    t0 = time.time()
    tex_seed = 0x504D5653 + (0 if (shard or world == 1) else 104729 * rank)
    if c4:
        inp, sp, c4_proj, c4_ids = c4_cluster(P, args, rank, world)
        args.views = len(c4_ids)
    else:
        inp, sp = P.synth_scene(args.views, args.width, args.height, level=args.level, supersample=2, nthreads=16,
                                seed=tex_seed)
    t_synth = time.time() - t0
    log(f"scene rendered ({args.views} x {args.width}x{args.height}) in {t_synth:.1f} s")
    t0 = time.time()
    scene = P.Scene(inp, device=local)
    t_scene = time.time() - t0
    t0 = time.time()
    seed_info = {"mode": args.seed_mode}
    if c4:
        seeds = c4_seeds(P, scene, sp, c4_proj, c4_ids, args.seeds * world)
        seed_info.update(mode="synthetic (cluster)", seed_patches=int(len(seeds)))
    elif args.seed_mode == "features":
        # CFindMatch::init's feature detection (findMatch.cpp:79-82, fcsize 16) and the seed phase
        # CSeed::run (findMatch.cpp:193) on the device
        points = [scene.detect_features(v) for v in range(args.views)]
        t_feat = time.time() - t0
        log(f"features: {sum(len(p) for p in points)} points in {t_feat:.1f} s; seed phase ...")
        seeds, sst = scene.seed_run(points)
        seed_info.update(points=int(sum(len(p) for p in points)), seed_patches=int(len(seeds)),
                         features_s=round(t_feat, 2), seed_s=round(time.time() - t0 - t_feat, 2),
                         trial=sst["trial"], passed=sst["pass"], candidates=sst["candidates"], refined=sst["refined"])
        del points
    else:
        cands = P.synth_candidates(sp, inp.projections, args.seeds, seed=rank_seed(0 if shard else rank))
        res, _ = scene.refine_batch(cands)
        seeds = P.patches_from_refined(res)
        seed_info.update(candidates=args.seeds, seed_patches=int(len(seeds)))
    t_seed = time.time() - t0
    log(f"{len(seeds)} seed patches ({args.seed_mode}) in {t_seed:.1f} s")
    ex = None
    if shard or (c4 and world > 1):  # native RCCL communicator (C++), records all-gathered device to device
        uid = [P.RcclExchange.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ex = P.RcclExchange(rank, world, uid[0], device=local)
        if shard:
            ex.attach(scene)
        else:
            ex.attach_cluster(scene, c4_ids)

    # One step = pmvs_run_loop: seeds up, 3 x (expand, filter), the model left in HBM (as the
    # refine inputs are, the result stays resident); its device digest (pmvs_loop_hash) checks that
    # every repetition gives the same model.  The final model's PCIe fetch (6.7 GB) runs after the
    # timed region and is reported as fetch_s.
    def step():
        n_kept, it_log = scene.run_loop(seeds, inp.threshold, iterations=args.iterations, wave=args.wave,
                                        min_candidates=args.min_candidates, fetch=False)
        return n_kept, it_log, f"{scene.loop_hash():016x}"

    import hashlib
    hashes = []
    for w in range(args.warmup):
        n_kept, _, h = step()
        log(f"warmup step {w + 1}/{args.warmup}: {n_kept} patches")
        hashes.append(h)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    logs = []
    n_last = 0
    for k in range(args.steps):
        n_last, it_log, h = step()
        logs.append((n_last, it_log))
        hashes.append(h)
        log(f"timed step {k + 1}/{args.steps}: {n_last} patches")
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tf = time.perf_counter()
    last = scene.loop_fetch(n_last)  # after the timed region
    fetch_s = time.perf_counter() - tf
    model_sha1 = hashlib.sha1(last.view(np.uint8)).hexdigest()

    def tot(key):
        return sum(it["expand"][key] for _, lg in logs for it in lg)
    added = tot("added")
    own_added = added if (not shard or rank == 0) else 0  # shard mode: one shared model
    refined, evals, tex_valid, refine_ms = tot("refined"), tot("evals"), tot("tex_valid"), tot("refine_ms")
    expand_s = tot("wall_ms") / 1e3
    filter_s = sum(it["filter"]["kernel_ms"] for _, lg in logs for it in lg) / 1e3
    (added_all, refined_all, evals_all), elapsed_max = reduce_over_ranks(dist, [own_added, refined, evals], elapsed,
                                                                         dev)
    launches = tot("refine_launches")
    traffic, traffic_launches, traffic_src = pmc_traffic("c3")
    # the dominant kernel: the split form, which runs the waves of >= 10k candidates; the
    # workgroup form's small batches (iterations 2-3) are reported beside it
    tv_s, ms_s, l_s = tot("tex_valid_small"), tot("refine_ms_small"), tot("refine_launches_small")
    roof = refine_roofline(tex_valid - tv_s, refine_ms - ms_s, launches - l_s, traffic, traffic_launches, traffic_src)
    small = refine_roofline(tv_s, ms_s, l_s, None, None, None)
    small["kernel"] = SMALL_KERNEL
    for k in ("traffic", "traffic_source", "traffic_launches", "bound", "peak", "unit"):
        small.pop(k)
    roof["small_batches"] = small

    result = None
    c2 = None
    if rank == 0 and not args.no_c2:
        c2 = c2_refine(P, args, dev, rank)
    if rank == 0:
        checks = model_checks(last, inp, hashes)
        checks["model_digest"] = checks.pop("model_hash")
        checks["model_hash"] = model_sha1  # sha1 of the fetched final model (the rounds' record format)
        del last
        cpu = parity = None
        first = logs[0][1]
        if not args.no_cpu_baseline and not shard and not c4:
            cpu, parity = loop_samples(P, scene, inp, seeds, args, [it["expand"]["added"] for it in first])
        result = {
            "metric": METRIC,
            "value": round(added_all / elapsed_max, 1),
            "unit": "refined patches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "vs_baseline": None,
            "dtype": "f32 (f64 optimizer)",
            "data": "synthetic (textured-sphere ring rendered by pmvs_synth_ring; seed model from "
                    + ("Harris/DoG features + the seed phase on the device)" if args.seed_mode == "features" else
                       "refined synthetic seed candidates)"),
            "config": {
                "workload": f"C3: {args.views}-view {args.width}x{args.height} synthetic ring, level {args.level}, "
                            f"full expand->optim->filter loop ({args.iterations} iterations) from "
                            + (f"the device seed phase's {len(seeds)} seed patches" if args.seed_mode == "features" else
                               f"{args.seeds} synthetic seed candidates")
                            + (", one scene sharded over all GPUs" if shard else
                               f", C4: cluster {rank} of a {args.c4_views_per_cluster * world}-view ring, boundary "
                               f"exchange over RCCL" if c4 else ", one cluster per GPU"),
                "views": args.views, "width": args.width, "height": args.height, "level": args.level,
                "seed_mode": args.seed_mode, "seed_patches": int(len(seeds)), "wave": args.wave,
                "min_candidates": args.min_candidates, "iterations": args.iterations, "wsize": 7, "csize": 2,
                "minImageNum": 3, "threshold": 0.7,
                "parallelism": (f"one shared scene, wave-sharded refine/findEmptyBlocks + target-owned filter x{world}"
                                if shard else f"CMVS clusters + RCCL boundary exchange x{world}" if c4 else
                                f"independent CMVS-style clusters, one {args.views}-view ring per GPU (weak scaling) x{world}"),
            },
            "ncc_evals_per_s": round(evals_all / elapsed_max, 1),
            "refined_candidates_per_s": round(refined_all / elapsed_max, 1),
            "model_patches": logs[0][0],
            "roofline": roof,
            "stage_s_per_step": {"expand": round(expand_s / args.steps, 3), "filter_device": round(filter_s / args.steps, 3),
                                 "refine_kernel": round(refine_ms / 1e3 / args.steps, 3)},
            "fetch_s": round(fetch_s, 3),  # the final model's D2H (pmvs_loop_fetch), outside the timed region
            "value_with_fetch": round(added_all / (elapsed_max + fetch_s * args.steps), 1),
            "iterations": [{"depth": it["depth"], "patches": it["patches"], "added": it["expand"]["added"],
                            "candidates": it["expand"]["candidates"], "waves": it["expand"]["waves"],
                            "expand_ms": round(it["expand"]["wall_ms"], 1),
                            "filter_ms": round(it["filter"]["kernel_ms"], 1),
                            "boundary": it["boundary"]} for it in first],
            "refine_c2": c2,
            "cpu_baseline": cpu,
            "parity_c3_first_waves": None if parity is None else all(p["ok"] for p in parity),
            "parity_c3_detail": parity,
            "checks": checks,
            "seed_phase": seed_info,
            "setup_s": {"synth": round(t_synth, 2), "scene": round(t_scene, 2), "seed": round(t_seed, 2)},
        }
        print(json.dumps(result), flush=True)
        if not checks["ok"]:
            print(f"bench.py: C3 model checks failed: {checks}", file=sys.stderr, flush=True)
        if parity is not None and not result["parity_c3_first_waves"]:
            print(f"bench.py: full-size parity against the oracle FAILED: {parity}", file=sys.stderr, flush=True)
            scene.close()
            sys.exit(3)
    scene.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
