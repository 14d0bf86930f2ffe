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
    cands = P.synth_candidates(sp, inp.projections, 64, seed=bench.rank_seed(rank))
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


def test_thread_exchange_allgather(product_lib):
    """pmvs_thread_allgather (the in-process exchange of sharded scenes): 3 threads, several
    rounds of different sizes, every rank receives every rank's bytes in rank order."""
    import ctypes as C
    import threading
    import pmvs_amd as P
    world, rounds = 3, 5
    ex = P.ThreadExchange(world)
    fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)(ex.endpoint(0)[0])
    got, errs = {}, []

    def work(r):
        try:
            for k in range(rounds):
                nb = 1000 * (k + 1) + 3
                send = np.full(nb, 16 * r + k, np.uint8)
                recv = np.zeros(nb * world, np.uint8)
                rc = fn(ex.endpoint(r)[1], send.ctypes.data, nb, recv.ctypes.data)
                got[(r, k)] = (rc, recv.reshape(world, nb)[:, 0].tolist(), bool((recv.reshape(world, nb) ==
                                                                                 recv.reshape(world, nb)[:, :1]).all()))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    ex.close()
    assert not errs
    for r in range(world):
        for k in range(rounds):
            rc, heads, uniform = got[(r, k)]
            assert rc == 0 and uniform
            assert heads == [16 * q + k for q in range(world)]


def _exchange_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cmvs-pmvs_amd")]
    import ctypes as C
    import torch.distributed as dist
    import pmvs_amd as P
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = P.DistExchange()
    res = []
    for nb in (17, 4096, 100003):
        send = (np.arange(nb) * (rank + 1) % 251).astype(np.uint8)
        recv = np.zeros(nb * world, np.uint8)
        rc = ex.fn(None, send.ctypes.data, nb, recv.ctypes.data)
        exp = np.concatenate([(np.arange(nb) * (q + 1) % 251).astype(np.uint8) for q in range(world)])
        res.append((rc, bool(np.array_equal(recv, exp))))
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


def test_dist_exchange_gloo_two_ranks(product_lib):
    """DistExchange (the pmvs_allgather_fn bench.py gives sharded scenes, RCCL on GPUs) over gloo:
    the C-callable callback all-gathers host buffers of several sizes in rank order."""
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_exchange_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        assert res[r] == [(0, True)] * 3
