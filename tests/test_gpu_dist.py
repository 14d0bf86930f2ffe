"""Multi-process tests of the distributed paths on one GPU.

* Two processes, one scene each on cuda:0, exchanging over torch.distributed/gloo through
  DistExchange (the host-buffer pmvs_allgather_fn): the wave-sharded loop (pmvs_scene_set_shard)
  equals the single-rank loop, and the cluster loop (pmvs_scene_set_cluster) equals the same two
  clusters run as threads in one process through the in-process exchange (whose semantics
  tests/test_gpu_cluster.py checks against the oracle).
* One process with torch's RCCL process group (backend "nccl") AND the library's own RCCL
  communicator (librccl.so.1 opened at run time): both all-gather and a sharded loop runs through
  the native communicator at world 1 -- they coexist in one process, as bench.py --mode shard uses
  them.
The children are separate programs (subprocess): RCCL and gloo process groups stay out of the test
runner, and each child's result is compared here.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COMMON = r"""
import hashlib, json, os, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "cmvs-pmvs_amd")]
import numpy as np
import pmvs_amd as P
def scene_and_seeds(views, ids=None, w=320, h=240, level=1, ncand=300):
    full, p = P.synth_scene(views, w, h, level=level, supersample=2, nthreads=8)
    cands = P.synth_candidates(p, full.projections, ncand, seed=7)
    if ids is None:
        g = P.Scene(full)
        r, _ = g.refine_batch(cands)
        return full, g, P.patches_from_refined(r)
    inp = P.SceneInputs(images=[full.images[i] for i in ids], projections=full.projections[ids], num_targets=len(ids),
                        level=full.level, csize=full.csize)
    loc = {v: k for k, v in enumerate(ids)}
    keep = [i for i, c in enumerate(cands) if int(c["images"][0]) in loc and int(c["images"][1]) in loc]
    cs = cands[keep].copy()
    for c in cs:
        c["images"][0] = loc[int(c["images"][0])]; c["images"][1] = loc[int(c["images"][1])]
    g = P.Scene(inp)
    r, _ = g.refine_batch(cs)
    return inp, g, P.patches_from_refined(r)
def digest(a):
    return hashlib.sha1(a.tobytes()).hexdigest()
"""

CHILD_GLOO = COMMON + r"""
import torch.distributed as dist
rank, world, mode = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), sys.argv[2]
dist.init_process_group("gloo", rank=rank, world_size=world)
ex = P.DistExchange()
kw = dict(wave=256, min_candidates=512)
if mode == "shard":
    inp, g, seeds = scene_and_seeds(6)
    ex.attach(g)
elif mode == "shard_ring50":  # a 50-view 1280x720 ring at level 0, the bench's C3 schedule
    inp, g, seeds = scene_and_seeds(50, None, 1280, 720, 0, 2000)
    ex.attach(g)
    kw = dict(wave=32768, min_candidates=131072)
else:
    ids = json.loads(sys.argv[3])[rank]
    inp, g, seeds = scene_and_seeds(8, ids)
    g.set_cluster(rank, world, ids, ex.fn, None)
out, log = g.run_loop(seeds, inp.threshold, **kw)
g.close()
print("RESULT", json.dumps({"rank": rank, "n": len(out), "digest": digest(out),
                            "sent": [it["boundary"]["sent"] for it in log]}), flush=True)
dist.barrier()
dist.destroy_process_group()
"""

CHILD_RCCL = COMMON + r"""
import torch, torch.distributed as dist
dist.init_process_group("nccl", rank=0, world_size=1)
t = torch.ones(4, device="cuda")
dist.all_reduce(t)
inp, g, seeds = scene_and_seeds(6)
uid = P.RcclExchange.unique_id()
ex = P.RcclExchange(0, 1, uid, device=0)
got = ex.allgather(b"pmvs-rccl")
ex.attach(g)
out, log = g.run_loop(seeds, inp.threshold, wave=256, min_candidates=512)
g.close()
ex.close()
t2 = torch.full((2,), 3.0, device="cuda")
dist.all_reduce(t2)
print("RESULT", json.dumps({"n": len(out), "digest": digest(out), "allgather": got.decode(),
                            "torch": float(t.sum()) + float(t2.sum())}), flush=True)
dist.destroy_process_group()
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _result(stdout):
    for line in stdout.splitlines():
        if line.startswith("RESULT "):
            return json.loads(line[len("RESULT "):])
    raise AssertionError(f"no result line:\n{stdout[-2000:]}")


def _run_gloo(mode, extra=()):
    world, port = 2, _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world))
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD_GLOO, ROOT, mode, *extra], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, err[-3000:]
        res.append(_result(out))
    return res


def _local(views, ids=None):
    import pmvs_amd as P
    full, p = P.synth_scene(views, 320, 240, level=1, supersample=2, nthreads=8)
    cands = P.synth_candidates(p, full.projections, 300, seed=7)
    return full, p, cands


@pytest.mark.timeout(600)
def test_two_process_sharded_loop_gloo(gpu_available):
    import pmvs_amd as P
    full, p, cands = _local(6)
    g = P.Scene(full)
    r, _ = g.refine_batch(cands)
    ref, _ = g.run_loop(P.patches_from_refined(r), full.threshold, wave=256, min_candidates=512)
    g.close()
    res = _run_gloo("shard")
    digest = hashlib.sha1(ref.tobytes()).hexdigest()
    assert [x["digest"] for x in res] == [digest, digest], (len(ref), res)


@pytest.mark.timeout(600)
def test_two_process_sharded_ring50_720p_gloo(gpu_available):
    """The owner-partitioned loop (wave-sharded refine / findEmptyBlocks / postProcess, target-owner
    filter stages) on a 50-view 1280x720 ring at level 0 with the bench's C3 schedule, two processes
    over gloo: both ranks' models equal the one-rank model byte for byte."""
    import pmvs_amd as P
    full, p = P.synth_scene(50, 1280, 720, level=0, supersample=2, nthreads=8)
    cands = P.synth_candidates(p, full.projections, 2000, seed=7)
    g = P.Scene(full)
    r, _ = g.refine_batch(cands)
    ref, _ = g.run_loop(P.patches_from_refined(r), full.threshold, wave=32768, min_candidates=131072)
    g.close()
    assert len(ref) > 50_000
    res = _run_gloo("shard_ring50")
    digest = hashlib.sha1(ref.tobytes()).hexdigest()
    assert [x["digest"] for x in res] == [digest, digest], (len(ref), res)


@pytest.mark.timeout(600)
def test_two_process_cluster_loop_gloo(gpu_available):
    import threading
    import pmvs_amd as P
    clusters = [[0, 1, 2, 3, 4], [4, 5, 6, 7, 0]]
    full, p, cands = _local(8)
    scenes, seeds, inps = [], [], []
    for ids in clusters:
        inp = P.SceneInputs(images=[full.images[i] for i in ids], projections=full.projections[ids],
                            num_targets=len(ids), level=full.level, csize=full.csize)
        loc = {v: k for k, v in enumerate(ids)}
        keep = [i for i, c in enumerate(cands) if int(c["images"][0]) in loc and int(c["images"][1]) in loc]
        cs = cands[keep].copy()
        for c in cs:
            c["images"][0] = loc[int(c["images"][0])]
            c["images"][1] = loc[int(c["images"][1])]
        g = P.Scene(inp)
        r, _ = g.refine_batch(cs)
        scenes.append(g)
        seeds.append(P.patches_from_refined(r))
        inps.append(inp)
    ex = P.ThreadExchange(2)
    out = [None, None]

    def work(r):
        scenes[r].set_cluster(r, 2, clusters[r], *ex.endpoint(r))
        out[r] = scenes[r].run_loop(seeds[r], inps[r].threshold, wave=256, min_candidates=512)

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for g in scenes:
        g.close()
    ex.close()
    assert all(o is not None for o in out)
    res = _run_gloo("cluster", (json.dumps(clusters),))
    for r in range(2):
        model, log = out[r]
        assert res[r]["digest"] == hashlib.sha1(model.tobytes()).hexdigest(), (r, len(model), res[r])
        assert res[r]["sent"] == [it["boundary"]["sent"] for it in log]
    assert sum(res[0]["sent"]) > 0


@pytest.mark.timeout(300)
def test_torch_rccl_and_native_rccl_coexist(gpu_available):
    import pmvs_amd as P
    full, p, cands = _local(6)
    g = P.Scene(full)
    r, _ = g.refine_batch(cands)
    ref, _ = g.run_loop(P.patches_from_refined(r), full.threshold, wave=256, min_candidates=512)
    g.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1")
    pr = subprocess.run([sys.executable, "-c", CHILD_RCCL, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert pr.returncode == 0, pr.stderr[-3000:]
    res = _result(pr.stdout)
    assert res["allgather"] == "pmvs-rccl"
    assert res["torch"] == 4.0 + 6.0
    assert res["digest"] == hashlib.sha1(ref.tobytes()).hexdigest()
