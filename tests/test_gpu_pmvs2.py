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
