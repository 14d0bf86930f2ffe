"""GPU parity of one expansion run (PMVS3::CExpand::run, expand.cpp:17-406) against the CPU
oracle (oracle/expand_oracle.h) on the same seed model: identical patch count, statistics, and
every field of every patch (new patches bit-for-bit: coord, normal, ncc, scales, images, grids,
vimages, vgrids; old patches' _flag).

The seed model is a set of refined patches of a synthetic ring (HIP refine path).  wave = 1 is
the reference's single-thread schedule; wave > 1 pops that many parents per round (DESIGN.md,
"Expansion"), and the oracle runs the same wave schedule."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("coord", "normal", "ncc", "dscale", "ascale", "tmp", "timages", "flag", "fix", "num_images",
          "num_vimages", "dflag")


def seed_model(P, g, inp, p, n, seed):
    cands = P.synth_candidates(p, inp.projections, n, seed=seed)
    r, _ = g.refine_batch(cands)
    return P.patches_from_refined(r)


def compare(out_g, al_g, st_g, out_o, al_o, st_o):
    assert len(out_g) == len(out_o), (len(out_g), len(out_o))
    for k in st_o:
        assert st_g[k] == st_o[k], (k, st_g[k], st_o[k])
    assert np.array_equal(al_g, al_o)
    for f in FIELDS:
        a, b = out_g[f], out_o[f]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        bad = np.nonzero((a != b).reshape(len(a), -1).any(1))[0]
        assert len(bad) == 0, (f, len(bad), bad[:8])
    for i in range(len(out_o)):
        n, m = out_o["num_images"][i], out_o["num_vimages"][i]
        assert np.array_equal(out_g["images"][i][:n], out_o["images"][i][:n]), i
        assert np.array_equal(out_g["grids"][i][:n], out_o["grids"][i][:n]), i
        assert np.array_equal(out_g["vimages"][i][:m], out_o["vimages"][i][:m]), i
        assert np.array_equal(out_g["vgrids"][i][:m], out_o["vgrids"][i][:m]), i


@pytest.mark.parametrize("depth,wave", [(1, 1), (2, 64), (1, 4096)], ids=["d1_w1", "d2_w64", "d1_w4096"])
def test_expand_matches_oracle(gpu_available, oracle_mod, depth, wave):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 300, 3)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
    out_g, al_g, st_g = g.expand_run(pa, wave=wave, cap=100000)
    out_o, al_o, st_o = o.expand_run(pa, wave=wave, cap=100000)
    g.close()
    o.close()
    assert st_g["added"] > 5 * len(pa)
    compare(out_g, al_g, st_g, out_o, al_o, st_o)


def test_expand_after_filter_with_dead_patches(gpu_available, oracle_mod):
    """Second expansion of a model a filter pass thinned (alive = keep), count threshold 2
    (the value after updateThreshold), including _fix patches."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 300, 4)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    m, al, _ = g.expand_run(pa, wave=256, cap=100000)
    assert (al == 1).all()
    m, keep, _ = g.filter_run(m)
    m["fix"][::97] = 1
    out_g, al_g, st_g = g.expand_run(m, alive=keep, wave=256, count_threshold=2, cap=200000)
    out_o, al_o, st_o = o.expand_run(m, alive=keep, wave=256, count_threshold=2, cap=200000)
    g.close()
    o.close()
    assert (keep == 0).any()
    compare(out_g, al_g, st_g, out_o, al_o, st_o)


def test_expand_capacity_error(gpu_available):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    pa = seed_model(P, g, inp, p, 100, 5)
    g.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    with pytest.raises(RuntimeError):
        g.expand_run(pa, wave=64, cap=len(pa) + 10)
    out, al, st = g.expand_run(pa[:0], wave=64, cap=16)
    assert len(out) == 0 and st["parents"] == 0
    g.close()


@pytest.mark.parametrize("wave,native", [(1, True), (512, True), (512, False)])
def test_full_loop_matches_oracle(gpu_available, oracle_mod, wave, native):
    """CFindMatch::run after the seed phase (findMatch.cpp:196-217): 3 x (expand, filter,
    updateThreshold) from refined seeds, first expansion with the seed phase's empty depth maps."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 200, 7)
    out_g, log_g = g.run_loop(pa, inp.threshold, wave=wave, native=native)
    out_o, log_o = o.run_loop(pa, inp.threshold, wave=wave)
    g.close()
    o.close()
    for a, b in zip(log_g, log_o):
        assert a["patches"] == b["patches"], (a, b)
        assert {k: v for k, v in a["expand"].items() if k not in P.ExpandStats.WORK} == b["expand"]
        assert [a["filter"][k] for k in ("removed_outside", "removed_exact", "removed_neighbor",
                                         "removed_groups")] == b["filter"]
    assert log_g[-1]["patches"] > 5 * len(pa)
    compare(out_g, np.ones(len(out_g), np.int32), {}, out_o, np.ones(len(out_o), np.int32), {})


def test_expand_device_growth_small_waves(gpu_available, oracle_mod):
    """wave = 8: the device patch arrays start at (model + 12 waves + 1024) and are regrown
    (contents kept) several times during the run; the result still equals the oracle's."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 120, 9)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    out_g, al_g, st_g = g.expand_run(pa, wave=8)
    out_o, al_o, st_o = o.expand_run(pa, wave=8, cap=200000)
    g.close()
    o.close()
    assert len(out_g) > 2 * (len(pa) + 12 * 8 + 1024)
    compare(out_g, al_g, st_g, out_o, al_o, st_o)


def run_sharded(P, inp, model, world, fn, expect_errors=False, **kw):
    """`world` scenes on GPU 0, one per thread, sharing one in-process all-gather (the same
    protocol bench.py runs with one process per GPU over RCCL)."""
    import threading
    ex = P.ThreadExchange(world)
    scenes = [P.Scene(inp) for _ in range(world)]
    for r, sc in enumerate(scenes):
        sc.set_shard(r, world, *ex.endpoint(r))
    res, errs = [None] * world, [None] * world

    def work(r):
        try:
            res[r] = fn(scenes[r], model, **kw)
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    hung = [r for r, t in enumerate(th) if t.is_alive()]
    assert not hung, f"ranks {hung} still blocked (exchange deadlock)"
    for sc in scenes:
        sc.close()
    ex.close()
    if expect_errors:
        return errs
    assert not any(errs), errs
    return res


@pytest.mark.parametrize("world,wave", [(2, 256), (3, 64)])
def test_sharded_expand_matches_single_rank(gpu_available, world, wave):
    """Sharded expansion: every rank's model after the run is bit-identical to
    the one-rank run with the same wave, and the ranks' refine shares add up to the candidates."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    pa = seed_model(P, g, inp, p, 300, 3)
    g.set_thresholds(inp.threshold, inp.threshold - 0.3, 2)
    ref, al_ref, st_ref = g.expand_run(pa, wave=wave)
    g.close()

    def fn(sc, model, **kw):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 2)
        return sc.expand_run(model, **kw)

    res = run_sharded(P, inp, pa, world, fn, wave=wave)
    for out, al, st in res:
        compare(out, al, {k: v for k, v in st.items() if k not in P.ExpandStats.WORK}, ref, al_ref,
                {k: v for k, v in st_ref.items() if k not in P.ExpandStats.WORK})
    assert sum(r[2]["refined"] for r in res) == st_ref["refined"]
    assert sum(r[2]["evals"] for r in res) == st_ref["evals"]
    assert all(r[2]["refined"] > 0 for r in res)


@pytest.mark.parametrize("where", ["b", "e", "a"])
def test_sharded_expand_rank_failure_fails_all_ranks(gpu_available, monkeypatch, where):
    """A failure on ONE rank of a sharded expansion (advice r01: an allocation failure between
    exchanges used to leave the peers blocked in the next all-gather) makes every rank return an
    error: injected on rank 1 at wave 2 before the wave (b), at its findEmptyBlocks candidate
    exchange (e), or right after its refine batch exchange (a)."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    pa = seed_model(P, g, inp, p, 300, 3)
    g.close()

    def fn(sc, model, **kw):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 2)
        return sc.expand_run(model, **kw)

    monkeypatch.setenv("PMVS_TEST_SHARD_FAIL", f"1:2:{where}")
    errs = run_sharded(P, inp, pa, 2, fn, expect_errors=True, wave=64)
    assert all(isinstance(e, P.PmvsError) for e in errs), errs


@pytest.mark.parametrize("where", ["f", "g", "s", "x"])
def test_sharded_loop_filter_failure_fails_all_ranks(gpu_available, monkeypatch, where):
    """The sharded loop's filter pass (owner-partitioned filterNeighbor, one flag all-gather):
    a failure on rank 1 before (f) or after (g) that exchange makes both ranks return an error;
    so does a local failure after the filter's last exchange (s) or after the expansion's last
    exchange (x) -- an asynchronous fault surfacing at that rank's stream synchronisation."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    pa = seed_model(P, g, inp, p, 200, 7)
    g.close()
    monkeypatch.setenv("PMVS_TEST_SHARD_FAIL", f"1:0:{where}")
    errs = run_sharded(P, inp, pa, 2, lambda sc, m, **kw: sc.run_loop(m, inp.threshold, **kw), expect_errors=True,
                       wave=512)
    assert all(isinstance(e, P.PmvsError) for e in errs), errs


def test_sharded_full_loop_matches_single_rank(gpu_available):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    pa = seed_model(P, g, inp, p, 200, 7)
    ref, log_ref = g.run_loop(pa, inp.threshold, wave=512)
    g.close()
    res = run_sharded(P, inp, pa, 2, lambda sc, m, **kw: sc.run_loop(m, inp.threshold, **kw), wave=512)
    for out, log in res:
        assert [x["patches"] for x in log] == [x["patches"] for x in log_ref]
        compare(out, np.ones(len(out), np.int32), {}, ref, np.ones(len(ref), np.int32), {})


@pytest.mark.parametrize("depth,softcap", [(1, None), (2, None), (1, "8"), (2, "8")],
                         ids=["d1", "d2", "d1_nb_rewalk", "d2_nb_rewalk"])
def test_expand_min_candidates_matches_oracle(gpu_available, oracle_mod, monkeypatch, depth, softcap):
    """Waves extended by further parent chunks until they hold min_candidates free directions
    (the schedule bench.py uses for C3): device and oracle run the same schedule.  PMVS_NB_SOFTCAP=8:
    findEmptyBlocks' and check()'s neighbour walks go through the NB_CAP_BIG re-walk."""
    import pmvs_amd as P
    if softcap is not None:  # findEmptyBlocks / depth >= 2 check() walks re-walked by the NB_CAP_BIG form
        monkeypatch.setenv("PMVS_NB_SOFTCAP", softcap)
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 300, 5)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, depth)
    out_g, al_g, st_g = g.expand_run(pa, wave=16, min_candidates=300)
    out_o, al_o, st_o = o.expand_run(pa, wave=16, min_candidates=300, cap=200000)
    g.close()
    o.close()
    assert st_o["waves"] < st_o["parents"] / 16
    compare(out_g, al_g, st_g, out_o, al_o, st_o)


def test_full_loop_min_candidates_matches_oracle(gpu_available, oracle_mod):
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = seed_model(P, g, inp, p, 200, 8)
    out_g, log_g = g.run_loop(pa, inp.threshold, wave=64, min_candidates=256)
    out_o, log_o = o.run_loop(pa, inp.threshold, wave=64, min_candidates=256)
    g.close()
    o.close()
    for a, b in zip(log_g, log_o):
        assert a["patches"] == b["patches"], (a, b)
        assert {k: v for k, v in a["expand"].items() if k not in P.ExpandStats.WORK} == b["expand"]
    compare(out_g, np.ones(len(out_g), np.int32), {}, out_o, np.ones(len(out_o), np.int32), {})
