"""CMVS cluster per GPU with the boundary exchange (pmvs_scene_set_cluster).

A 12-view ring is split into three overlapping clusters the way CMVS writes them (ske.dat: each
cluster a list of target images, neighbouring clusters sharing images; bundle.cpp:1465-1485,
genOption.cpp:73-108).  Three cluster scenes run pmvs_run_loop on one GPU, one thread each, their
exchanges going through the in-process all-gather (ThreadExchange).  The same three loops are
emulated with the CPU oracle -- expand and filter per cluster and iteration, and between
iterations the boundary exchange restated in numpy: every cluster's patches registered in a target
image another cluster also targets are inserted into the other clusters as the reference's
readPatches inserts another run's patches (patchOrganizerS.cpp:133-197: image numbers mapped to
indexes, _vimages cleared, setGrids), fixed and never expanded (fix = PMVS_FIX_FOREIGN).  Each
cluster's final model must equal the emulation's patch for patch.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROD = dict(wave=256, min_candidates=1024)
CLUSTERS = [[0, 1, 2, 3, 4], [4, 5, 6, 7, 8], [8, 9, 10, 11, 0]]  # global image numbers (targets)


def _cluster_scene(P, full, ids):
    return P.SceneInputs(images=[full.images[i] for i in ids], projections=full.projections[ids],
                         num_targets=len(ids), level=full.level, csize=full.csize)


def _cluster_seeds(P, g, cands_global, ids):
    """Seed-path candidates of the full ring whose two images are in this cluster, as local indexes."""
    loc = {v: k for k, v in enumerate(ids)}
    keep = [i for i, c in enumerate(cands_global) if int(c["images"][0]) in loc and int(c["images"][1]) in loc]
    cands = cands_global[keep].copy()
    for c in cands:
        c["images"][0] = loc[int(c["images"][0])]
        c["images"][1] = loc[int(c["images"][1])]
    r, _ = g.refine_batch(cands)
    return P.patches_from_refined(r)


def _boundary(P, model, ids, shared, gw, gh):
    """This cluster's patches registered in a shared target (in-grid target entries)."""
    tnum = len(ids)
    sel = []
    for i, q in enumerate(model):
        if q["fix"] == P.FIX_FOREIGN:
            continue
        for k in range(q["num_images"]):
            t = int(q["images"][k])
            gx, gy = int(q["grids"][k][0]), int(q["grids"][k][1])
            if t < tnum and shared[t] and 0 <= gx < gw[t] and 0 <= gy < gh[t]:
                sel.append(i)
                break
    return model[sel]


def _insert(P, o, records, src_ids, ids, gw, gh):
    """readPatches-style insertion of another cluster's records into this cluster (oracle setGrids)."""
    loc = {v: k for k, v in enumerate(ids)}
    tnum = len(ids)
    out = []
    for q in records:
        gl = [src_ids[int(q["images"][k])] for k in range(q["num_images"])]
        if gl[0] not in loc:
            continue
        mapped = [loc[v] for v in gl if v in loc]
        p = np.zeros(1, P.PATCH_DTYPE)[0]
        for f in ("coord", "normal", "ncc", "dscale", "ascale"):
            p[f] = q[f]
        p["flag"], p["fix"], p["dflag"], p["num_vimages"], p["tmp"] = 1, P.FIX_FOREIGN, 0, 0, 0.0
        p["num_images"] = len(mapped)
        p["images"][:len(mapped)] = mapped
        p["timages"] = sum(1 for v in mapped if v < tnum)
        p = o.set_grids(np.array([p], P.PATCH_DTYPE))[0]
        reg = any(int(p["images"][k]) < tnum and 0 <= p["grids"][k][0] < gw[p["images"][k]]
                  and 0 <= p["grids"][k][1] < gh[p["images"][k]] for k in range(len(mapped)))
        if reg:
            out.append(p)
    return np.array(out, P.PATCH_DTYPE) if out else np.zeros(0, P.PATCH_DTYPE)


def _emulate(P, O, inps, seeds, iterations=3):
    G = len(CLUSTERS)
    os_ = [O.OracleScene(inp) for inp in inps]
    grid = []
    for inp in inps:
        gw = [(im.shape[1] // (1 << inp.level) + inp.csize - 1) // inp.csize for im in inp.images]
        gh = [(im.shape[0] // (1 << inp.level) + inp.csize - 1) // inp.csize for im in inp.images]
        grid.append((gw, gh))
    tsets = [set(c) for c in CLUSTERS]
    shared = [[any(v in tsets[q] for q in range(G) if q != r) for v in CLUSTERS[r]] for r in range(G)]
    models = [s.copy() for s in seeds]
    ncc = np.float32(inps[0].threshold)
    before = np.float32(ncc - np.float32(0.3))
    cthr, depth, stats = 4, 1, []
    for t in range(iterations):
        for r in range(G):
            o = os_[r]
            o.set_thresholds(float(ncc), float(before), depth)
            m, _, _ = o.expand_run(models[r], wave=PROD["wave"], count_threshold=cthr, cap=1 << 20,
                                   after_seeds=(t == 0), min_candidates=PROD["min_candidates"])
            m, keep, _ = o.filter_run(m)
            models[r] = m[keep == 1]
        if t + 1 < iterations:
            own = [m[m["fix"] != P.FIX_FOREIGN] for m in models]
            bnd = [_boundary(P, own[r], CLUSTERS[r], shared[r], *grid[r]) for r in range(G)]
            new = []
            for r in range(G):
                parts = [own[r]]
                for q in range(G):
                    if q != r and len(bnd[q]):
                        parts.append(_insert(P, os_[r], bnd[q], CLUSTERS[q], CLUSTERS[r], *grid[r]))
                new.append(np.concatenate(parts))
            stats.append([len(b) for b in bnd])
            models = new
        ncc = np.float32(ncc - np.float32(0.05))
        before = np.float32(before - np.float32(0.05))
        cthr, depth = 2, depth + 1
    for o in os_:
        o.close()
    return [m[m["fix"] != P.FIX_FOREIGN] for m in models], stats


@pytest.mark.timeout(900)
def test_cluster_exchange_matches_oracle_emulation(gpu_available, oracle_mod):
    import pmvs_amd as P
    from test_gpu_parity_matrix import _same_patches
    full, p = P.synth_scene(12, 320, 240, level=1, supersample=2, nthreads=8)
    cands = P.synth_candidates(p, full.projections, 600, seed=13)
    inps = [_cluster_scene(P, full, ids) for ids in CLUSTERS]
    scenes = [P.Scene(inp) for inp in inps]
    seeds = [_cluster_seeds(P, g, cands, ids) for g, ids in zip(scenes, CLUSTERS)]
    assert all(len(s) > 0 for s in seeds)
    ex = P.ThreadExchange(len(CLUSTERS))
    res, errs = [None] * len(CLUSTERS), [None] * len(CLUSTERS)

    def work(r):
        try:
            scenes[r].set_cluster(r, len(CLUSTERS), CLUSTERS[r], *ex.endpoint(r))
            res[r] = scenes[r].run_loop(seeds[r], inps[r].threshold, cap=1 << 20, **PROD)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(len(CLUSTERS))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "cluster exchange deadlock"
    for g in scenes:
        g.close()
    ex.close()
    assert not any(errs), errs
    emu, bstats = _emulate(P, oracle_mod, inps, seeds)
    print(f"boundary patches per exchange: {bstats}; final models {[len(m) for m in emu]}")
    assert all(sum(b) > 0 for b in bstats)  # the exchange moved patches
    for r, ((out, log), ref) in enumerate(zip(res, emu)):
        assert [it["boundary"]["sent"] for it in log[:-1]] == [b[r] for b in bstats], (r, log)
        assert all(it["boundary"]["inserted"] > 0 for it in log[:-1]), log
        assert len(out) == len(ref), (r, len(out), len(ref))
        assert out.tobytes() == ref.tobytes() or _same_patches(out, ref), r


def test_cluster_exchange_single_rank_is_a_no_op(gpu_available):
    """world = 1 turns the exchange off: the loop equals the plain loop."""
    import pmvs_amd as P
    full, p = P.synth_scene(6, 320, 240, level=1, supersample=2, nthreads=8)
    g = P.Scene(full)
    cands = P.synth_candidates(p, full.projections, 150, seed=3)
    r, _ = g.refine_batch(cands)
    seeds = P.patches_from_refined(r)
    ref, _ = g.run_loop(seeds, full.threshold, **PROD)
    g.set_cluster(0, 1, list(range(6)))
    out, log = g.run_loop(seeds, full.threshold, **PROD)
    g.close()
    assert out.tobytes() == ref.tobytes()
    assert all(it["boundary"]["sent"] == 0 for it in log)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("where", ["x", "s"], ids=["after_expansion", "after_filter"])
def test_cluster_local_failure_fails_all_ranks(gpu_available, monkeypatch, where):
    """A failure local to one cluster rank (injected after its expansion, or after its filter pass,
    as an asynchronous fault surfacing at the stream synchronisation would) is announced on the
    cluster channel: every rank returns an error and none is left blocked in the boundary
    exchange or the final loop header (the expansion / filter exchanges of a cluster
    scene run at world 1, so their failures are never known to the peers)."""
    import pmvs_amd as P
    full, p = P.synth_scene(12, 320, 240, level=1, supersample=2, nthreads=8)
    cands = P.synth_candidates(p, full.projections, 300, seed=13)
    inps = [_cluster_scene(P, full, ids) for ids in CLUSTERS]
    scenes = [P.Scene(inp) for inp in inps]
    seeds = [_cluster_seeds(P, g, cands, ids) for g, ids in zip(scenes, CLUSTERS)]
    monkeypatch.setenv("PMVS_TEST_SHARD_FAIL", f"1:0:{where}")
    ex = P.ThreadExchange(len(CLUSTERS))
    errs = [None] * len(CLUSTERS)

    def work(r):
        try:
            scenes[r].set_cluster(r, len(CLUSTERS), CLUSTERS[r], *ex.endpoint(r))
            scenes[r].run_loop(seeds[r], inps[r].threshold, cap=1 << 20, **PROD)
        except P.PmvsError as e:
            errs[r] = str(e)

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(len(CLUSTERS))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=200)
    assert not any(t.is_alive() for t in th), "a rank is blocked after a peer's local failure"
    for g in scenes:
        g.close()
    ex.close()
    print(errs)
    assert all(errs), errs
    assert "injected" in errs[1]


def test_cluster_setup_validation_fails_all_ranks(gpu_available):
    """pmvs_scene_set_cluster validates after the collective: a rank with a bad image list (a
    duplicate image number) makes every rank fail, instead of returning before the all-gather and
    leaving its peers blocked in it."""
    import pmvs_amd as P
    full, p = P.synth_scene(8, 160, 120, level=1, supersample=1, nthreads=8)
    ids = [[0, 1, 2, 3, 4], [4, 5, 6, 7, 0]]
    inps = [_cluster_scene(P, full, c) for c in ids]
    scenes = [P.Scene(inp) for inp in inps]
    bad = [list(ids[0]), [4, 5, 6, 6, 0]]  # rank 1 names image 6 twice
    ex = P.ThreadExchange(2)
    errs = [None, None]

    def work(r):
        try:
            scenes[r].set_cluster(r, 2, bad[r], *ex.endpoint(r))
        except P.PmvsError as e:
            errs[r] = str(e)

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "cluster setup deadlock"
    for g in scenes:
        g.close()
    ex.close()
    assert errs[0] and errs[1], errs
    assert "twice" in errs[1] and "rank 1" in errs[0], errs
