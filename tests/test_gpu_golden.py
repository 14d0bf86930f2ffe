"""GPU parity against the committed golden vectors (tests/golden/*.npz): the HIP path through
the C-ABI must reproduce them bit-for-bit (pyramids by CRC, textures, my_f values, refined
patch records)."""
import glob
import os
import zlib

import numpy as np
import pytest

from pmvs_cases import bits

pytestmark = pytest.mark.gpu
# scene goldens (c1, ring8); expand_dirs / features / seeds / isneighbor / organizer.npz hold other reference vectors
GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith(("expand_dirs", "features", "seeds", "isneighbor", "organizer")))


@pytest.fixture(scope="module", params=GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def gscene(request, gpu_available):
    import pmvs_amd as P
    g = dict(np.load(request.param))
    views, width, height, level, csize = (int(v) for v in g["params"])
    inp, p = P.synth_scene(views, width, height, level=level, csize=csize, supersample=2)
    s = P.Scene(inp)
    yield g, inp, s
    s.close()


def test_pyramid_golden(gscene):
    g, inp, s = gscene
    crc = np.array([[zlib.crc32(s.get_level(v, lv).tobytes()) for lv in range(g["pyramid_crc"].shape[1])]
                    for v in range(len(inp.images))], np.uint32)
    assert np.array_equal(crc, g["pyramid_crc"])


def test_grab_tex_golden(gscene):
    g, inp, s = gscene
    tex, valid = s.grab_tex(g["tex_query"])
    assert np.array_equal(valid, g["tex_valid"])
    assert np.array_equal(bits(tex), bits(g["tex"]))


def test_my_f_golden(gscene):
    g, inp, s = gscene
    f, st = s.incc_eval(g["eval_query"])
    assert np.array_equal(bits(f), bits(g["eval_f"])), np.flatnonzero(bits(f) != bits(g["eval_f"]))[:10]


def test_refine_golden(gscene):
    g, inp, s = gscene
    out, st = s.refine_batch(g["refine_in"])
    exp = g["refine_out"]
    assert np.array_equal(out["status"], exp["status"])
    acc = exp["status"] == 0
    for f in ("refine_code", "evals", "num_images", "timages"):
        assert np.array_equal(out[f][acc], exp[f][acc]), f
    for f in ("coord", "normal", "ncc", "dscale", "ascale", "tmp"):
        assert np.array_equal(bits(out[f][acc]), bits(exp[f][acc])), f
    for i in np.flatnonzero(acc):
        n = exp["num_images"][i]
        assert np.array_equal(out["images"][i][:n], exp["images"][i][:n])
        assert np.array_equal(out["grids"][i][:n], exp["grids"][i][:n])
    got = [st[k] for k in ("accepted", "fail_pre", "fail_post", "refine_failed", "evals", "tex_valid")]
    assert got == list(g["refine_stats"])
