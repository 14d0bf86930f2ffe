"""GPU parity of one filter pass (PMVS3::CFilter::run, filter.cpp:13-27: filterOutside,
filterExact, filterNeighbor, filterSmallGroups with the depth-map / vimages rebuilds between
them) against the CPU oracle (oracle/filter_oracle.h) on the same patch set: identical keep
flags, removal counts, image lists, cells, timages and vimages.

Patch sets: refined patches of a dense synthetic ring (the HIP refine path, bit-exact with the
oracle), plus injected outliers (copies displaced towards the camera with low NCC, which
filterOutside must remove) and a few fixed patches (_fix = 1, never removed)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def make_patch_set(P, g, inp, p, n_cand, seed, outliers=0.02, fixed=0.01):
    cands = P.synth_candidates(p, inp.projections, n_cand, seed=seed)
    r, _ = g.refine_batch(cands)
    pa = P.patches_from_refined(r)
    rng = np.random.default_rng(seed)
    k = int(len(pa) * outliers)
    if k:
        src = pa[rng.choice(len(pa), k, replace=False)].copy()
        for q in src:
            ref = int(q["images"][0])
            cam = np.asarray(inp.projections[ref], np.float64)
            # optical centre of the reference camera: null vector of P
            M = cam[:, :3]
            c = -np.linalg.solve(M, cam[:, 3])
            d = c - q["coord"][:3].astype(np.float64)
            d /= np.linalg.norm(d)
            q["coord"][:3] = (q["coord"][:3] + d * 25.0 * q["dscale"]).astype(np.float32)
            q["ncc"] = np.float32(inp.threshold + 0.02)
        pa = np.concatenate([pa, src])
    fx = rng.random(len(pa)) < fixed
    pa["fix"][fx] = 1
    return pa


def compare(out_g, keep_g, st_g, out_o, keep_o, counts_o):
    assert np.array_equal(keep_g, keep_o), int((keep_g != keep_o).sum())
    assert [st_g["removed_outside"], st_g["removed_exact"], st_g["removed_neighbor"], st_g["removed_groups"]] == \
        list(counts_o)
    for f in ("timages", "num_images", "num_vimages", "flag"):
        assert np.array_equal(out_g[f], out_o[f]), f
    for i in range(len(out_o)):
        n, m = out_o["num_images"][i], out_o["num_vimages"][i]
        assert np.array_equal(out_g["images"][i][:n], out_o["images"][i][:n]), i
        assert np.array_equal(out_g["grids"][i][:n], out_o["grids"][i][:n]), i
        assert np.array_equal(out_g["vimages"][i][:m], out_o["vimages"][i][:m]), i
        assert np.array_equal(out_g["vgrids"][i][:m], out_o["vgrids"][i][:m]), i


@pytest.mark.parametrize("cfg", [dict(views=8, w=960, h=540, level=1, n=100000, seed=5),
                                 dict(views=6, w=640, h=480, level=2, n=4000, seed=6, csize=4)],
                         ids=["ring8_level1", "ring6_level2_c4"])
def test_filter_pass_matches_oracle(gpu_available, oracle_mod, cfg):
    import pmvs_amd as P
    opts = {"csize": cfg["csize"]} if "csize" in cfg else {}
    inp, p = P.synth_scene(cfg["views"], cfg["w"], cfg["h"], level=cfg["level"], supersample=2, nthreads=16, **opts)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = make_patch_set(P, g, inp, p, cfg["n"], cfg["seed"])
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    out_g, keep_g, st_g = g.filter_run(pa)
    out_o, keep_o, counts_o = o.filter_run(pa)
    g.close()
    o.close()
    assert st_g["removed_outside"] > 0 and st_g["kept"] > len(pa) // 2
    assert (keep_g[pa["fix"] == 1] == 1).mean() > 0.5
    compare(out_g, keep_g, st_g, out_o, keep_o, counts_o)


def test_filter_depth0_and_empty(gpu_available, oracle_mod):
    """At depth 0 isVisible accepts every in-grid cell (patchOrganizerS.cpp:506)."""
    import pmvs_amd as P
    inp, p = P.synth_scene(6, 480, 360, level=1, supersample=2)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = make_patch_set(P, g, inp, p, 8000, 9, outliers=0.0, fixed=0.0)
    out_g, keep_g, st_g = g.filter_run(pa)
    out_o, keep_o, counts_o = o.filter_run(pa)
    compare(out_g, keep_g, st_g, out_o, keep_o, counts_o)
    out, keep, st = g.filter_run(pa[:0])
    assert len(keep) == 0 and st["kept"] == 0
    g.close()
    o.close()


@pytest.mark.parametrize("cap,qwaves,qlds,softcap", [("0", "0", "96", None), ("20000", "0", "96", None),
                                                      ("-1", "1", "0", None), ("-1", "0", "12", None),
                                                      ("-1", "0", "160", None), ("-1", "0", "96", "8")],
                         ids=["all_in_wave", "mixed", "lane_grid_stride", "lds_and_lane", "lds_160", "nb_rewalk"])
def test_filter_quad_deferral_paths(gpu_available, oracle_mod, monkeypatch, cap, qwaves, qlds, softcap):
    """filterNeighbor's quadric fits run after the neighbour walk -- eight lanes per fit with the
    rows in LDS (quad_qr_kernel + quad_solve_kernel) up to PMVS_QUAD_LDS_ROWS rows, one lane per fit
    (quad_lane_kernel) above -- or inside the walk's wavefront when the deferred-row buffer is
    full; PMVS_QUAD_ROWS caps that buffer so both paths (and a mix) meet the oracle.
    PMVS_QUAD_WAVES_PER_CU = 1 caps the lane kernel's grid, so each lane fits several jobs
    (the grid-stride path); PMVS_QUAD_LDS_ROWS = 12 splits the fits between the two kernels.
    PMVS_NB_SOFTCAP = 8: the neighbour walk's overflow path (the NB_CAP_BIG re-walk)."""
    import pmvs_amd as P
    if cap != "-1":
        monkeypatch.setenv("PMVS_QUAD_ROWS", cap)
    monkeypatch.setenv("PMVS_QUAD_WAVES_PER_CU", qwaves)
    monkeypatch.setenv("PMVS_QUAD_LDS_ROWS", qlds)
    if softcap:  # the NB_CAP walk holds 8 neighbours: nearly every patch is re-walked by the NB_CAP_BIG form
        monkeypatch.setenv("PMVS_NB_SOFTCAP", softcap)
    inp, p = P.synth_scene(8, 960, 540, level=1, supersample=2, nthreads=16)
    g = P.Scene(inp)
    o = oracle_mod.OracleScene(inp)
    pa = make_patch_set(P, g, inp, p, 30000, 11)
    for sc in (g, o):
        sc.set_thresholds(inp.threshold, inp.threshold - 0.3, 1)
    out_g, keep_g, st_g = g.filter_run(pa)
    out_o, keep_o, counts_o = o.filter_run(pa)
    g.close()
    o.close()
    compare(out_g, keep_g, st_g, out_o, keep_o, counts_o)
