#!/usr/bin/env python3
"""bench.py -- MI355X PMVS2 refine throughput (BASELINE.json metric), one JSON line on rank 0.

Workload (BASELINE.json configs[1], "C2"): a synthetic 8-view 1920x1080 textured-sphere ring,
level 1, csize 2, wsize 7, minImageNum 3, threshold 0.7; 100,000 seed-path candidates per GPU
(CSeed::initialMatchSub shape: images = [most frontal view, next view], depth perturbed,
normal tilted <= 10 deg).  One step = preProcess -> refinePatch (BOBYQA, <=1000 my_f evals)
-> postProcess over the whole batch on the device (candidates and results resident in HBM).

value = refined (accepted) patches/s over all ranks; also reported: NCC evals/s.
roofline: algorithmic bytes = 588 B x valid textures per my_f evaluation over
the refine kernel's HIP-event time, against 8 TB/s HBM.
cpu_baseline: the oracle (CPU restatement, std::thread pool) on a bounded sample on this host.

Multi-GPU (weak scaling): `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`;
each rank owns one GPU and its own candidate batch; no data-path collective (the path shards
by candidate); only barriers and the max-over-ranks time reduction.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--candidates", type=int, default=100000)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-filter", action="store_true", help="skip the filter-pass side measurement")
    return ap.parse_args()


def pmc_traffic(args):
    """HBM bytes per refine launch from the committed rocprofv3 PMC summary (tools/gpu_round.sh +
    tools/summarize_profiles.py; FETCH_SIZE x2 per MI355X_MICROARCH.md + WRITE_SIZE) when it was
    measured on this same default workload; otherwise null."""
    if (args.candidates, args.views, args.width, args.height, args.level) != (100000, 8, 1920, 1080, 1):
        return None, None
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for f in reversed(files):
        d = json.load(open(f))
        for k, v in d.get("kernels", {}).items():
            if "refine_v2_kernel" in k and k.endswith(os.environ.get("PMVS_REFINE_CONFIG_NAME", "<7, 16, 8>")):
                return int(v["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


def rank_candidate_seed(rank: int) -> int:
    """Each rank refines its own candidate shard (weak scaling, no data-path exchange)."""
    return 0x5EED + 7919 * rank


def reduce_over_ranks(dist, counts, elapsed, device):
    """SUM the per-rank counters and MAX the per-rank timed-region length over all ranks (the
    only collectives of the benchmark).  Works with nccl (RCCL) on GPUs and gloo on CPUs."""
    import torch
    totals = torch.tensor([float(c) for c in counts], dtype=torch.float64, device=device)
    tmax = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return totals.tolist(), tmax.item()


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

    # ---- scene (identical on every rank) and this rank's candidates
    t0 = time.time()
    inp, sp = P.synth_scene(args.views, args.width, args.height, level=args.level, supersample=2, nthreads=16)
    t_synth = time.time() - t0
    scene = P.Scene(inp, device=local)
    cands = P.synth_candidates(sp, inp.projections, args.candidates, seed=rank_candidate_seed(rank))
    nbytes_in = cands.nbytes
    d_in = torch.from_numpy(cands.view(np.uint8)).to(dev)
    d_out = torch.empty(args.candidates * P.REFINED_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def step():
        scene.refine_batch_device(d_in.data_ptr(), args.candidates, d_out.data_ptr())
        return scene.sync()

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(step())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    accepted = sum(s["accepted"] for s in stats)
    evals = sum(s["evals"] for s in stats)
    tex_valid = sum(s["tex_valid"] for s in stats)
    kernel_ms = [s["refine_ms"] for s in stats]
    stage_ms = {k: round(float(np.mean([s[k] for s in stats])), 3) for k in ("pre_ms", "refine_ms", "post_ms")}
    prof = {k: sum(s[k] for s in stats) for k in ("opt_cycles", "objective_cycles", "rounds", "chunks")}
    phase = np.sum([s["prof"] for s in stats], axis=0)
    phase_names = ("refill", "step", "publish", "chunk_setup", "gather", "normalize", "dot", "reduce")
    (accepted_all, evals_all, texv_all, cand_all), elapsed_max = reduce_over_ranks(
        dist, [accepted, evals, tex_valid, args.candidates * args.steps], elapsed, dev)

    # ---- roofline of the dominant kernel (refine_v2_kernel), per launch, HIP-event timed on the
    # scene stream (events recorded right before and after that launch)
    avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
    bytes_per_launch = tex_valid / args.steps * BYTES_PER_TEXTURE
    achieved = bytes_per_launch / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0

    # ---- side measurement: one CFilter::run pass (depth 1) over this rank's refined patches
    filt = None
    if not args.no_filter:
        res = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=P.REFINED_DTYPE)
        patches = P.patches_from_refined(res)
        scene.set_thresholds(0.7, 0.4, 1)
        t0 = time.perf_counter()
        _, keep, fst = scene.filter_run(patches)
        tf = time.perf_counter() - t0
        scene.set_thresholds(0.7, 0.4, 0)
        filt = {"patches": int(len(patches)), "kept": int(fst["kept"]), "device_ms": round(fst["kernel_ms"], 3),
                "wall_ms": round(tf * 1e3, 3), "patches_per_s": round(len(patches) / (fst["kernel_ms"] / 1e3), 1),
                "removed": [int(fst[k]) for k in ("removed_outside", "removed_exact", "removed_neighbor",
                                                  "removed_groups")]}
    traffic, traffic_src = pmc_traffic(args)
    result = None
    if rank == 0:
        # ---- CPU baseline (oracle restatement on this host, bounded sample)
        cpu = None
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as O
            o = O.OracleScene(inp)
            threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            done = acc_cpu = 0
            chunk = 2000
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds and done < len(cands):
                r, st = o.refine_batch(cands[done:done + chunk], nthreads=threads)
                done += len(r)
                acc_cpu += st["accepted"]
            tc = time.perf_counter() - t0
            o.close()
            cpu = {"value": round(acc_cpu / tc, 1), "unit": "refined patches/s", "cores": threads, "kind": "port",
                   "sample": f"first {done} of the {args.candidates} rank-0 candidates, oracle/liboracle.so "
                             f"(CPU restatement, std::thread pool), {tc:.1f} s"}
        result = {
            "metric": METRIC,
            "value": round(accepted_all / elapsed_max, 1),
            "unit": "refined patches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (f64 optimizer)",
            "data": "synthetic (textured-sphere ring rendered by pmvs_synth_ring; seeded candidates)",
            "config": {
                "workload": f"C2: {args.views}-view {args.width}x{args.height} synthetic ring, level {args.level}, "
                            f"{args.candidates} seed candidates per GPU, preProcess->refinePatch->postProcess",
                "candidates_per_gpu": args.candidates, "views": args.views, "width": args.width,
                "height": args.height, "level": args.level, "wsize": 7, "csize": 2, "minImageNum": 3,
                "parallelism": f"candidate-sharded x{world}",
            },
            "ncc_evals_per_s": round(evals_all / elapsed_max, 1),
            "accepted_fraction": round(accepted_all / cand_all, 4),
            "evals_per_candidate": round(evals_all / cand_all, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": "refine_v2_kernel<7,16,8>", "kernel_ms_avg": round(avg_kernel_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "traffic_source": traffic_src},
            "stage_ms": stage_ms,
            "filter_pass": filt,
            "cpu_baseline": cpu,
            "setup_s": {"synth": round(t_synth, 2)},
            "refine_profile": {"optimizer_cycle_frac": round(prof["opt_cycles"] / max(1, prof["opt_cycles"] + prof["objective_cycles"]), 4),
                               "rounds": prof["rounds"], "chunks": prof["chunks"],
                               "phase_frac": {k: round(float(v) / max(1.0, float(phase.sum())), 4) for k, v in zip(phase_names, phase)},
                               "config": int(os.environ.get("PMVS_REFINE_CONFIG", "1608")),
                               "waves_per_cu": int(os.environ.get("PMVS_REFINE_WAVES_PER_CU", "4"))},
            "input_bytes_resident": nbytes_in,
        }
        print(json.dumps(result), flush=True)
    scene.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
