"""BASELINE.json configs[3] (C4) at its full per-GPU size, on one GPU (C5: tests/test_gpu_c5.py).

C4 -- CMVS clusters of a 4K ring, one per GPU, boundary patches exchanged after every iteration
(pmvs_scene_set_cluster).  Three overlapping clusters of a 75-view 3840x2160 ring
(25 targets each plus 2 views shared with each neighbour, as `bench.py --mode c4` splits the ring)
run as three threads on this GPU, their exchanges through the in-process all-gather:
  * the full 3-iteration loop of every cluster: the bench's size-independent model checks and a
    non-empty boundary exchange;
  * bounded parity of the whole cluster loop, exchange included: every iteration's expansion
    stopped after its first waves (PMVS_EXPAND_MAX_WAVES), the filter passes and the exchanges run
    in full, against the CPU oracle's expand / filter per cluster with the exchange restated in
    numpy (the semantics tests/test_gpu_cluster.py checks on a small ring) -- record for record.

"""
import os
import sys
import threading

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


def _grid_wh(inp):
    gw = np.array([((im.shape[1] >> inp.level) + inp.csize - 1) // inp.csize for im in inp.images], np.int64)
    gh = np.array([((im.shape[0] >> inp.level) + inp.csize - 1) // inp.csize for im in inp.images], np.int64)
    return gw, gh


def _in_grid_targets(model, tnum, gw, gh, mask_t=None):
    """[n, K] bool: list entry k is a target image (optionally one with mask_t[t]) and its cell is in the grid."""
    k = np.arange(model["images"].shape[1])[None, :]
    im = model["images"].astype(np.int64)
    sel = (k < model["num_images"][:, None]) & (im < tnum)
    t = np.where(sel, im, 0)
    gx, gy = model["grids"][..., 0].astype(np.int64), model["grids"][..., 1].astype(np.int64)
    sel &= (gx >= 0) & (gx < gw[t]) & (gy >= 0) & (gy < gh[t])
    if mask_t is not None:
        sel &= mask_t[t]
    return sel


def boundary(P, model, tnum, shared, gw, gh):
    """cluster_exchange's boundary set: own patches registered in a shared target cell."""
    own = model["fix"] != P.FIX_FOREIGN
    return model[own & _in_grid_targets(model, tnum, gw, gh, np.asarray(shared, bool)).any(axis=1)]


def insert(P, o, records, src_ids, ids, tnum, gw, gh):
    """boundary_insert_kernel restated: another cluster's records in this cluster (image numbers ->
    indexes, dropping views it lacks; reference image required; _vimages cleared; setGrids by the
    oracle; kept when registered in one of this cluster's target cells), fixed and never expanded."""
    if len(records) == 0:
        return np.zeros(0, P.PATCH_DTYPE)
    loc = {v: i for i, v in enumerate(ids)}
    out = np.zeros(len(records), P.PATCH_DTYPE)
    ok = np.zeros(len(records), bool)
    for i, q in enumerate(records):
        gl = [src_ids[int(x)] for x in q["images"][:q["num_images"]]]
        if gl[0] not in loc:
            continue
        mapped = [loc[v] for v in gl if v in loc]
        p = out[i]
        for f in ("coord", "normal", "ncc", "dscale", "ascale"):
            p[f] = q[f]
        p["flag"], p["fix"] = 1, P.FIX_FOREIGN
        p["num_images"] = len(mapped)
        p["images"][:len(mapped)] = mapped
        p["timages"] = sum(1 for v in mapped if v < tnum)
        ok[i] = True
    out = out[ok]
    if len(out) == 0:
        return out
    out = o.set_grids(out)
    return out[_in_grid_targets(out, tnum, gw, gh).any(axis=1)]


def ring_clusters(views_per_cluster, world, overlap):
    V = views_per_cluster * world
    return [[(views_per_cluster * r - overlap + k) % V for k in range(views_per_cluster + 2 * overlap)]
            for r in range(world)]


@pytest.fixture(scope="module")
def c4_setup(gpu_available):
    import pmvs_amd as P
    world, vpc, ov = 3, 25, 2
    clusters = ring_clusters(vpc, world, ov)
    full, sp = P.synth_scene(vpc * world, 3840, 2160, level=0, supersample=2, nthreads=16)
    cands = P.synth_candidates(sp, full.projections, 5000 * world, seed=0x5EED)
    inps = [P.SceneInputs(images=[full.images[i] for i in ids], projections=full.projections[ids], num_targets=len(ids),
                          level=0) for ids in clusters]
    del full
    scenes = [P.Scene(inp) for inp in inps]
    seeds = []
    for g, ids in zip(scenes, clusters):
        loc = {v: k for k, v in enumerate(ids)}
        keep = [i for i in range(len(cands)) if int(cands["images"][i][0]) in loc and int(cands["images"][i][1]) in loc]
        cs = cands[keep].copy()
        cs["images"][:, 0] = [loc[int(v)] for v in cs["images"][:, 0]]
        cs["images"][:, 1] = [loc[int(v)] for v in cs["images"][:, 1]]
        r, _ = g.refine_batch(cs)
        seeds.append(P.patches_from_refined(r))
    yield P, clusters, inps, scenes, seeds
    for g in scenes:
        g.close()


def _run_clusters(P, clusters, inps, scenes, seeds, **kw):
    world = len(clusters)
    ex = P.ThreadExchange(world)
    res, errs = [None] * world, [None] * world

    def work(r):
        try:
            scenes[r].set_cluster(r, world, clusters[r], *ex.endpoint(r))
            res[r] = scenes[r].run_loop(seeds[r], inps[r].threshold, wave=32768, min_candidates=131072, **kw)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th), "cluster exchange deadlock"
    ex.close()
    for g in scenes:
        g.set_cluster(0, 1, list(range(len(g.inputs.images))))
    assert not any(errs), errs
    return res


@pytest.mark.timeout(900)
def test_c4_full_loop_model_checks(c4_setup):
    import bench
    P, clusters, inps, scenes, seeds = c4_setup
    res = _run_clusters(P, clusters, inps, scenes, seeds)
    for r, (model, log) in enumerate(res):
        checks = bench.model_checks(model, inps[r], ["x"])
        print(f"C4 cluster {r}: seeds {len(seeds[r])}, patches {[it['patches'] for it in log]}, boundary "
              f"{[(it['boundary']['sent'], it['boundary']['inserted']) for it in log]}, checks {checks}")
        assert checks["ok"], (r, checks)
        assert checks["sphere_residual_p99"] < 0.01, checks
        assert len(model) > 100 * len(seeds[r])
        assert all(it["boundary"]["sent"] > 0 and it["boundary"]["inserted"] > 0 for it in log[:-1]), log
        assert model["fix"].max() != P.FIX_FOREIGN  # foreign patches never returned


@pytest.mark.timeout(900)
def test_c4_bounded_loop_with_exchange_matches_oracle(c4_setup, oracle_mod):
    from bench import patch_mismatches
    P, clusters, inps, scenes, seeds = c4_setup
    waves, iterations = 2, 2
    res = _run_clusters(P, clusters, inps, scenes, seeds, iterations=iterations, max_waves=waves)
    # the oracle: per cluster expand (first `waves` waves) + filter, then the exchange in numpy
    G = len(clusters)
    os_ = [oracle_mod.OracleScene(inp) for inp in inps]
    grids = [_grid_wh(inp) for inp in inps]
    tsets = [set(c) for c in clusters]
    shared = [[any(v in tsets[q] for q in range(G) if q != r) for v in clusters[r]] for r in range(G)]
    models = [s.copy() for s in seeds]
    ncc = np.float32(inps[0].threshold)
    before = np.float32(ncc - np.float32(0.3))
    cthr, depth, sent = 4, 1, []
    oracle_mod.lib().oracle_set_threads(_threads())
    for t in range(iterations):
        for r in range(G):
            o = os_[r]
            o.set_thresholds(float(ncc), float(before), depth)
            m, _, _ = o.expand_run(models[r], wave=32768, count_threshold=cthr, cap=len(models[r]) + 600000,
                                   after_seeds=(t == 0), min_candidates=131072, nthreads=_threads(), max_waves=waves)
            m, keep, _ = o.filter_run(m)
            models[r] = m[keep == 1]
        if t + 1 < iterations:
            own = [m[m["fix"] != P.FIX_FOREIGN] for m in models]
            bnd = [boundary(P, own[r], len(clusters[r]), shared[r], *grids[r]) for r in range(G)]
            sent.append([len(b) for b in bnd])
            models = [np.concatenate([own[r]] + [insert(P, os_[r], bnd[q], clusters[q], clusters[r], len(clusters[r]),
                                                        *grids[r]) for q in range(G) if q != r]) for r in range(G)]
        ncc = np.float32(ncc - np.float32(0.05))
        before = np.float32(before - np.float32(0.05))
        cthr, depth = 2, depth + 1
    for o in os_:
        o.close()
    want = [m[m["fix"] != P.FIX_FOREIGN] for m in models]
    print(f"C4 bounded loop: boundary sent {sent}, final {[len(m) for m in want]}")
    assert all(sum(s) > 0 for s in sent)
    for r, ((out, log), ref) in enumerate(zip(res, want)):
        assert [it["boundary"]["sent"] for it in log[:-1]] == [s[r] for s in sent], (r, log)
        assert patch_mismatches(out, ref) == 0, r
