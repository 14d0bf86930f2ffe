"""End-to-end GPU test of the pmvs2 executable (reference pmvs.cpp:7-63): a C1-style dataset tree
(visualize/*.ppm, txt/*.txt, masks/*.pgm, option file) is run through cmvs-pmvs_amd/pmvs2, and its
.patch / .pset / .ply outputs are compared byte for byte with the CPU oracle's pipeline on the same
inputs (features -> CSeed -> 3 x (expand, filter) -> collectPatches(1) order -> the reference-pinned
writers).  `CPU 1` selects the reference's single-thread schedule; `CPU 8` the wave schedule."""
import os
import subprocess

import numpy as np
import pytest

from test_gpu_parity_matrix import blob_masks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMVS2 = os.path.join(ROOT, "cmvs-pmvs_amd", "pmvs2")


def write_contour(path, proj):
    with open(path, "w") as f:
        f.write("CONTOUR\n")
        for row in proj:
            f.write(" ".join(repr(float(v)) for v in row) + "\n")


def make_dataset(root, views, w, h, level, csize, cpu, masks=False, numbers=None):
    import pmvs_amd as P
    inp, p = P.synth_scene(views, w, h, level=level, csize=csize, supersample=2)
    numbers = numbers or list(range(views))
    for d in ("visualize", "txt", "models", "masks"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    mk = blob_masks(views, h, w, 4, keep=0.93) if masks else None
    for v, num in enumerate(numbers):
        with open(os.path.join(root, "visualize", "%08d.ppm" % num), "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (w, h) + np.ascontiguousarray(inp.images[v]).tobytes())
        write_contour(os.path.join(root, "txt", "%08d.txt" % num), inp.projections[v])
        if masks:
            with open(os.path.join(root, "masks", "%08d.pgm" % num), "wb") as f:
                f.write(b"P5\n%d %d\n255\n" % (w, h) + mk[v].tobytes())
    with open(os.path.join(root, "option-0000"), "w") as f:
        f.write(f"level {level}\ncsize {csize}\nthreshold 0.7\nwsize 7\nminImageNum 3\nCPU {cpu}\n"
                f"useVisData 0\nsequence -1\ntimages {len(numbers)} " + " ".join(map(str, numbers)) + "\noimages 0\n")
    return numbers


def oracle_outputs(root, cpu, out_prefix):
    """The oracle pipeline on the dataset as pmvs2 reads it (same files, same parsers)."""
    import pmvs_amd as P
    import pyoracle as O
    opt = P.options_load(root + "/", "option-0000")
    nums = opt["timages"] + opt["oimages"]
    imgs = [P.image_load(os.path.join(root, "visualize", "%08d.ppm" % n)) for n in nums]
    proj = np.stack([P.camera_load(os.path.join(root, "txt", "%08d.txt" % n)) for n in nums])
    mpath = [os.path.join(root, "masks", "%08d.pgm" % n) for n in nums]
    masks = [P.mask_load(m) for m in mpath] if all(os.path.exists(m) for m in mpath) else None
    inp = P.SceneInputs(images=imgs, projections=proj, num_targets=len(opt["timages"]), level=opt["level"],
                        csize=opt["csize"], wsize=opt["wsize"], min_image_num=opt["min_image_num"],
                        threshold=opt["threshold"], masks=masks)
    g = P.Scene(inp)
    pts = [g.detect_features(v) for v in range(len(nums))]
    o = O.OracleScene(inp)
    seeds, _ = o.seed_run(pts)
    wave, minc = (1, 0) if cpu == 1 else (32768, 131072)
    model, _ = o.run_loop(seeds, inp.threshold, wave=wave, min_candidates=minc)
    # collectPatches(1) order: lowest target image holding the patch, its cell there, model order
    tnum = inp.num_targets
    gw = [((imgs[t].shape[1] >> opt["level"]) + opt["csize"] - 1) // opt["csize"] for t in range(tnum)]
    keys = []
    for i, q in enumerate(model):
        ims = list(q["images"][:q["num_images"]])
        ts = [(t, k) for k, t in enumerate(ims) if t < tnum]
        t, k = min(ts)
        keys.append(((t << 40) + int(q["grids"][k][1]) * gw[t] + int(q["grids"][k][0]), i))
    model = model[[i for _, i in sorted(keys)]]
    fields = np.concatenate([model["coord"], model["normal"], model["ncc"].reshape(-1, 1),
                             model["dscale"].reshape(-1, 1), model["ascale"].reshape(-1, 1)], 1).astype(np.float32)
    images = [[nums[x] for x in q["images"][:q["num_images"]]] for q in model]
    vimages = [[nums[x] for x in q["vimages"][:q["num_vimages"]]] for q in model]
    P.write_patches(out_prefix + ".patch", fields, images, vimages)
    P.write_pset(out_prefix + ".pset", fields)
    cols = g.patch_colors(model["coord"], [list(q["images"][:q["num_images"]]) for q in model])
    P.write_ply(out_prefix + ".ply", fields, cols)
    g.close()
    o.close()
    return len(seeds), len(model)


@pytest.mark.parametrize("cpu,masks", [(1, False), (8, True)])
def test_pmvs2_c1_matches_oracle(gpu_available, tmp_path, cpu, masks):
    root = str(tmp_path / "pmvs")
    make_dataset(root, 3, 640, 480, 2, 4, cpu, masks=masks, numbers=[0, 3, 7])
    r = subprocess.run([PMVS2, root + "/", "option-0000", "PATCH", "PSET"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ns, nm = oracle_outputs(root, cpu, str(tmp_path / "oracle"))
    assert nm > ns > 0
    for ext in (".patch", ".pset", ".ply"):
        got = open(os.path.join(root, "models", "option-0000" + ext), "rb").read()
        want = open(str(tmp_path / "oracle") + ext, "rb").read()
        assert got == want, ext


def _load_cluster(root, option):
    import pmvs_amd as P
    opt = P.options_load(root + "/", option)
    nums = opt["timages"] + opt["oimages"]
    imgs = [P.image_load(os.path.join(root, "visualize", "%08d.ppm" % n)) for n in nums]
    proj = np.stack([P.camera_load(os.path.join(root, "txt", "%08d.txt" % n)) for n in nums])
    inp = P.SceneInputs(images=imgs, projections=proj, num_targets=len(opt["timages"]), level=opt["level"],
                        csize=opt["csize"], wsize=opt["wsize"], min_image_num=opt["min_image_num"],
                        threshold=opt["threshold"])
    return opt, nums, inp


def _write_collect_order(P, model, inp, opt, nums, path):
    """writePatches2's collectPatches(1) order (lowest target image holding the patch, its cell,
    model order) and the reference-pinned .patch writer, as pmvs2 writes it."""
    tnum = inp.num_targets
    gw = [((inp.images[t].shape[1] >> opt["level"]) + opt["csize"] - 1) // opt["csize"] for t in range(tnum)]
    keys = []
    for i, q in enumerate(model):
        ts = [(int(t), k) for k, t in enumerate(q["images"][:q["num_images"]]) if t < tnum]
        t, k = min(ts)
        keys.append(((t << 40) + int(q["grids"][k][1]) * gw[t] + int(q["grids"][k][0]), i))
    model = model[[i for _, i in sorted(keys)]]
    fields = np.concatenate([model["coord"], model["normal"], model["ncc"].reshape(-1, 1),
                             model["dscale"].reshape(-1, 1), model["ascale"].reshape(-1, 1)], 1).astype(np.float32)
    P.write_patches(path, fields, [[nums[x] for x in q["images"][:q["num_images"]]] for q in model],
                    [[nums[x] for x in q["vimages"][:q["num_vimages"]]] for q in model])


@pytest.mark.timeout(600)
def test_pmvs2_two_rank_cluster_job_matches_thread_exchange(gpu_available, tmp_path):
    """The drop-in pipeline's multi-rank mode (genOption --gpus N): two pmvs2
    processes, one per overlapping CMVS cluster option file (genOption.cpp:73-108), form one job
    (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT) and exchange boundary patches after every loop
    iteration -- here over the TCP channel, both ranks on this one GPU (RCCL allows one rank per
    device).  Each rank's .patch must equal, byte for byte, the same two clusters run in one
    process with the in-process thread exchange (features, seed phase and loop on the device)."""
    import socket
    import threading
    import pmvs_amd as P
    root = str(tmp_path / "pmvs")
    make_dataset(root, 8, 320, 240, 1, 2, 8, numbers=list(range(8)))
    clusters = [[0, 1, 2, 3, 4], [4, 5, 6, 7, 0]]
    for r, t in enumerate(clusters):
        with open(os.path.join(root, "option-%04d" % r), "w") as f:
            f.write("level 1\ncsize 2\nthreshold 0.7\nwsize 7\nminImageNum 3\nCPU 8\nuseVisData 0\nsequence -1\n"
                    f"timages {len(t)} " + " ".join(map(str, t)) + "\noimages 0\n")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PMVS_EXCHANGE="tcp")
        procs.append(subprocess.Popen([PMVS2, root + "/", "option-%04d" % r, "PATCH"], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=400) for p in procs]
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, (r, e[-3000:])
    sent = [int(line.split("boundary sent ")[1].split()[0]) for _, e in outs for line in e.splitlines()
            if "boundary sent" in line]
    assert sum(sent) > 0, [e[-1500:] for _, e in outs]
    # the same job in one process: two scenes, two threads, the in-process exchange
    loaded = [_load_cluster(root, "option-%04d" % r) for r in range(2)]
    scenes = [P.Scene(inp) for _, _, inp in loaded]
    seeds = []
    for g, (_, nums, _) in zip(scenes, loaded):
        pts = [g.detect_features(v) for v in range(len(nums))]
        seeds.append(g.seed_run(pts)[0])
    ex = P.ThreadExchange(2)
    res, errs = [None, None], [None, None]

    def work(r):
        try:
            scenes[r].set_cluster(r, 2, loaded[r][1], *ex.endpoint(r))
            res[r] = scenes[r].run_loop(seeds[r], loaded[r][2].threshold, wave=32768, min_candidates=131072)[0]
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th) and not any(errs), errs
    for g in scenes:
        g.close()
    ex.close()
    for r in range(2):
        opt, nums, inp = loaded[r]
        want = str(tmp_path / ("thread-%d.patch" % r))
        _write_collect_order(P, res[r], inp, opt, nums, want)
        got = open(os.path.join(root, "models", "option-%04d.patch" % r), "rb").read()
        assert got == open(want, "rb").read(), r


@pytest.mark.timeout(300)
def test_pmvs2_job_rank_failure_ends_the_job(gpu_available, tmp_path):
    """A rank that fails before the loop (here: its option file names an image that does not
    exist) exits; its peer sees the closed connection and exits with an error instead of blocking."""
    import socket
    root = str(tmp_path / "pmvs")
    make_dataset(root, 4, 160, 120, 1, 2, 8, numbers=list(range(4)))
    for r, t in enumerate([[0, 1, 2], [2, 3, 9]]):  # image 9 is missing
        with open(os.path.join(root, "option-%04d" % r), "w") as f:
            f.write("level 1\ncsize 2\nCPU 8\ntimages %d %s\noimages 0\n" % (len(t), " ".join(map(str, t))))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([PMVS2, root + "/", "option-%04d" % r],
                              env=dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PMVS_EXCHANGE="tcp"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=200) for p in procs]
    assert procs[1].returncode != 0 and procs[0].returncode != 0, [e[-800:] for _, e in outs]
    assert "another rank" in outs[0][1], outs[0][1][-800:]
