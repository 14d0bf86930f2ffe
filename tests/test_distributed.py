"""Multi-process (world_size 2, gloo, CPU) test of bench.py's distributed path: each rank owns a
disjoint candidate shard (rank-seeded), processes it independently (here with the CPU oracle,
test-only), and the only collectives are the SUM of counters and the MAX of the timed region."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cmvs-pmvs_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import bench
    import pmvs_amd as P
    import pyoracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp, sp = P.synth_scene(4, 160, 120, level=1, supersample=1)
    cands = P.synth_candidates(sp, inp.projections, 64, seed=bench.rank_candidate_seed(rank))
    o = O.OracleScene(inp)
    r, st = o.refine_batch(cands, nthreads=1)
    o.close()
    elapsed = 0.5 + rank  # distinct per rank: the reduction must return the max
    totals, tmax = bench.reduce_over_ranks(dist, [st["accepted"], st["evals"], st["tex_valid"], len(cands)],
                                           elapsed, "cpu")
    out[rank] = (st["accepted"], st["evals"], st["tex_valid"], totals, tmax, cands["coord"][:4].tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_reduction(product_lib, oracle_mod):
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    acc = sum(res[r][0] for r in range(world))
    ev = sum(res[r][1] for r in range(world))
    tv = sum(res[r][2] for r in range(world))
    for r in range(world):
        totals, tmax = res[r][3], res[r][4]
        assert totals == [acc, ev, tv, 64 * world]
        assert tmax == 1.5
    assert res[0][5] != res[1][5]  # disjoint, rank-seeded shards
    assert acc > 0
