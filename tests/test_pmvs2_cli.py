"""CPU tests of the pmvs2 / genOption executables and the image-input surface (SURVEY.md §8(b)
external boundary, §8(f) f3/f4):
  * genOption (cmvs-pmvs_amd/genOption) against the reference's own genOption.cpp compiled
    unmodified into oracle/_ref: identical option files and pmvs.sh for the same ske.dat;
  * JPEG input against libjpeg 9's own djpeg (the image's /opt/conda/bin/djpeg, libjpeg defaults
    = CImg's load_jpeg path of CImage::readAnyImage);
  * P5 / P4 mask readers and CImage::setEdge (numpy restatement in the same float order);
  * pmvs2 usage / error exits (no GPU needed)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cmvs-pmvs_amd")
REF_GENOPTION = os.path.join(ROOT, "oracle", "_ref", "genOption")


def write_ske(path, clusters, inum=40):
    with open(path, "w") as f:
        f.write(f"SKE\n{inum} {len(clusters)}\n")
        for t, o in clusters:
            f.write(f"{len(t)} {len(o)}\n" + " ".join(map(str, t)) + "\n" + " ".join(map(str, o)) + "\n")


@pytest.mark.parametrize("args", [[], ["2"], ["0", "1", "0.55", "9", "2", "16"]])
def test_genoption_matches_reference(product_lib, tmp_path, args):
    if not os.path.exists(REF_GENOPTION):
        pytest.skip("oracle/_ref/genOption not built (reference absent)")
    clusters = [(list(range(0, 12)), [12, 13, 14]), (list(range(12, 25)), [3, 4]), ([30], [])]
    outs = []
    for tool in (os.path.join(PKG, "genOption"), REF_GENOPTION):
        d = tmp_path / os.path.basename(os.path.dirname(tool))
        d.mkdir()
        write_ske(d / "ske.dat", clusters)
        subprocess.run([tool, str(d) + "/"] + args, check=True)
        outs.append({f: (d / f).read_bytes() for f in sorted(os.listdir(d)) if f != "ske.dat"})
    assert outs[0] == outs[1]
    assert len(outs[0]) == len(clusters) + 1


def test_genoption_gpu_script(product_lib, tmp_path):
    write_ske(tmp_path / "ske.dat", [([0, 1], [2]), ([2, 3], []), ([4], [5]), ([6], [])])
    subprocess.run([os.path.join(PKG, "genOption"), str(tmp_path) + "/", "--gpus", "2"], check=True)
    s = (tmp_path / "pmvs_gpus.sh").read_text()
    # clusters in jobs of 2 ranks: {0, 1} on GPUs 0, 1, then {2, 3}; each job's ranks exchange
    assert "MASTER_PORT=$((PORT+0)) WORLD_SIZE=2 RANK=0 LOCAL_RANK=0 pmvs2 pmvs/ option-0000 &" in s
    assert "MASTER_PORT=$((PORT+0)) WORLD_SIZE=2 RANK=1 LOCAL_RANK=1 pmvs2 pmvs/ option-0001 &" in s
    assert "MASTER_PORT=$((PORT+1)) WORLD_SIZE=2 RANK=1 LOCAL_RANK=1 pmvs2 pmvs/ option-0003 &" in s
    assert s.index("option-0001") < s.index("wait $p") < s.index("option-0002")
    assert (tmp_path / "option-0003").exists() and (tmp_path / "pmvs.sh").exists()
    # a job of one rank for an odd cluster count
    write_ske(tmp_path / "ske.dat", [([0, 1], [2]), ([2, 3], []), ([4], [5])])
    subprocess.run([os.path.join(PKG, "genOption"), str(tmp_path) + "/", "--gpus", "2"], check=True)
    s = (tmp_path / "pmvs_gpus.sh").read_text()
    assert "WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 pmvs2 pmvs/ option-0002 &" in s
    assert subprocess.run(["sh", "-n", str(tmp_path / "pmvs_gpus.sh")]).returncode == 0


def test_tcp_allgather_processes(product_lib, tmp_path):
    """pmvs_tcp (the multi-rank pmvs2 job's host channel): three processes all-gather their blocks in
    rank order, a size mismatch fails the exchange on every rank, and a rank that exits makes its
    peers' next exchange fail instead of blocking."""
    import socket
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    prog = f"""
import ctypes as C, sys
sys.path.insert(0, {os.path.join(ROOT, 'cmvs-pmvs_amd')!r})
import pmvs_amd as P
lib = P.load_library()
rank, world = int(sys.argv[1]), 3
h = C.c_void_p()
assert lib.pmvs_tcp_create(rank, world, b"127.0.0.1", {port}, 20000, C.byref(h)) == 0, lib.pmvs_last_error()
send = bytes([rank + 1] * 5)
recv = C.create_string_buffer(15)
assert lib.pmvs_tcp_allgather(h, send, 5, recv) == 0
assert recv.raw == bytes([1] * 5 + [2] * 5 + [3] * 5), recv.raw
n = 4 if rank == 2 else 5                      # rank 2 sends a different size: every rank fails
assert lib.pmvs_tcp_allgather(h, send, n, recv) == -1
assert lib.pmvs_tcp_allgather(h, send, 5, recv) == 0  # and the channel still works afterwards
if rank == 1:
    sys.exit(0)                                 # rank 1 leaves: the others' next exchange fails
r = lib.pmvs_tcp_allgather(h, send, 5, recv)
assert r == -1, r
print("ok", rank)
"""
    f = tmp_path / "tcp_rank.py"
    f.write_text(prog)
    ps = [subprocess.Popen([sys.executable, str(f), str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
          for r in range(3)]
    outs = [p.communicate(timeout=60) for p in ps]
    for r, (p, (o, e)) in enumerate(zip(ps, outs)):
        assert p.returncode == 0, (r, o, e)
    assert "ok 0" in outs[0][0] and "ok 2" in outs[2][0]


def test_tcp_allgather_status_write_failure(product_lib, tmp_path):
    """pmvs_tcp's dead-peer path (round-5 advisor): rank 0's status write to rank 2 fails after rank 1
    was already told success (PMVS_TEST_TCP_FAIL=2:2 on rank 0: its second exchange).  Rank 1 must still get its payload and
    the failing commit word instead of waiting for bytes that never come; every rank returns -1, and
    the next exchange fails on every live rank too (rank 2's channel is closed) -- nobody blocks."""
    import socket
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    prog = f"""
import ctypes as C, sys
sys.path.insert(0, {os.path.join(ROOT, 'cmvs-pmvs_amd')!r})
import pmvs_amd as P
lib = P.load_library()
rank, world = int(sys.argv[1]), 3
h = C.c_void_p()
assert lib.pmvs_tcp_create(rank, world, b"127.0.0.1", {port}, 20000, C.byref(h)) == 0, lib.pmvs_last_error()
send = bytes([rank + 1] * 5)
recv = C.create_string_buffer(15)
assert lib.pmvs_tcp_allgather(h, send, 5, recv) == 0
r = lib.pmvs_tcp_allgather(h, send, 5, recv)   # rank 0 fails its status write to rank 2
assert r == -1, (rank, r)
if rank != 2:
    r = lib.pmvs_tcp_allgather(h, send, 5, recv)   # rank 2 is cut off: the next exchange fails as well
    assert r == -1, (rank, r)
print("ok", rank)
"""
    f = tmp_path / "tcp_fail.py"
    f.write_text(prog)
    env = dict(os.environ)
    env.pop("PMVS_TEST_TCP_FAIL", None)
    ps = [subprocess.Popen([sys.executable, str(f), str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           env=dict(env, PMVS_TEST_TCP_FAIL="2:2") if r == 0 else env) for r in range(3)]
    outs = [p.communicate(timeout=60) for p in ps]
    for r, (p, (o, e)) in enumerate(zip(ps, outs)):
        assert p.returncode == 0, (r, o, e)
        assert f"ok {r}" in o


def test_jpeg_matches_libjpeg(product_lib, tmp_path):
    import pmvs_amd as P
    cjpeg, djpeg = shutil.which("cjpeg") or "/opt/conda/bin/cjpeg", shutil.which("djpeg") or "/opt/conda/bin/djpeg"
    if not (os.path.exists(cjpeg) and os.path.exists(djpeg)):
        pytest.skip("libjpeg tools absent")
    rng = np.random.default_rng(3)
    img = (rng.random((61, 83, 3)) * 255).astype(np.uint8)
    img[20:40, 10:50] = [200, 30, 90]
    ppm = tmp_path / "a.ppm"
    ppm.write_bytes(b"P6\n83 61\n255\n" + img.tobytes())
    jpg = tmp_path / "a.jpg"
    with open(jpg, "wb") as f:
        subprocess.run([cjpeg, "-quality", "85", str(ppm)], stdout=f, check=True)
    ref = subprocess.run([djpeg, "-pnm", str(jpg)], stdout=subprocess.PIPE, check=True).stdout
    ref_px = np.frombuffer(ref[-83 * 61 * 3:], np.uint8).reshape(61, 83, 3)
    got = P.image_load(str(jpg))
    assert got.shape == (61, 83, 3)
    assert np.array_equal(got, ref_px)
    assert np.array_equal(P.image_load(str(ppm)), img)


def test_mask_readers(product_lib, tmp_path):
    import pmvs_amd as P
    m = (np.arange(7 * 5) % 3 == 0).astype(np.uint8) * 200
    (tmp_path / "m.pgm").write_bytes(b"P5\n# c\n7 5\n255\n" + m.tobytes())
    assert np.array_equal(P.mask_load(str(tmp_path / "m.pgm")), m.reshape(5, 7))
    bits = (np.arange(7 * 5) % 4 == 1).astype(np.uint8)  # 1 = black (outside)
    packed = np.packbits(np.concatenate([bits, np.zeros(5, np.uint8)]))
    (tmp_path / "m.pbm").write_bytes(b"P4\n7 5\n" + packed.tobytes())
    assert np.array_equal(P.mask_load(str(tmp_path / "m.pbm")), np.where(bits == 1, 0, 255).astype(np.uint8).reshape(5, 7))


def test_set_edge_restatement(product_lib):
    """CImage::setEdge (image.cpp:407-460) restated in numpy with the same float32 operation order."""
    import pmvs_amd as P
    rng = np.random.default_rng(9)
    img = np.repeat(np.repeat((np.arange(52) * 2 + 20).astype(np.uint8)[None, :, None], 40, 0), 3, 2)
    img = (img + (rng.random(img.shape) * 6).astype(np.uint8)).astype(np.uint8)
    img[:, 26:] += 90
    H, W = img.shape[:2]
    a = np.zeros((H, W), np.float32)
    im = img.astype(np.int32)
    for i in range(3):
        d0 = np.abs(im[1:-1, 2:, i] - im[1:-1, :-2, i])
        d1 = np.abs(im[2:, 1:-1, i] - im[:-2, 1:-1, i])
        a[1:-1, 1:-1] += (d0 * d0).astype(np.float32)
        a[1:-1, 1:-1] += (d1 * d1).astype(np.float32)
    sigma2 = np.float32(18.0)
    flt = np.array([np.float32(np.exp(np.float64(np.float32(-i * i) / sigma2))) for i in range(-6, 7)], np.float32)

    def smooth(x, axis):
        out = np.zeros_like(x)
        n = x.shape[axis]
        for idx in range(n):
            acc = np.zeros(x.shape[1 - axis], np.float32)
            den = np.float32(0)
            for j in range(-6, 7):
                t = idx + j
                if t < 0 or t >= n:
                    continue
                acc = acc + flt[j + 6] * (x[t] if axis == 0 else x[:, t])
                den = np.float32(den + flt[j + 6])
            if axis == 0:
                out[idx] = acc / den
            else:
                out[:, idx] = acc / den
        return out

    s = smooth(smooth(a, 0), 1)
    thr = np.float32(5.0)
    nt = np.float32(np.float32(np.float32(thr * thr) * np.float32(13)) * np.float32(13)) / np.float32(3.0)
    want = np.where(nt < s, 255, 0).astype(np.uint8)
    got = P.set_edge(img, 5.0)
    assert np.array_equal(got, want)
    assert 0 < (got == 255).sum() < got.size


def test_pmvs2_usage(product_lib):
    r = subprocess.run([os.path.join(PKG, "pmvs2")], capture_output=True, text=True)
    assert r.returncode == 1
    assert "prefix option_file [Optional export]" in r.stderr and "PATCH PSET" in r.stderr


def test_pmvs2_missing_option_file(product_lib, tmp_path):
    r = subprocess.run([os.path.join(PKG, "pmvs2"), str(tmp_path) + "/", "nope"], capture_output=True, text=True)
    assert r.returncode == 1
    assert "pmvs2: option file" in r.stderr
