"""Native RCCL communicator (cmvs-pmvs_amd/csrc/pmvs_rccl.cpp): created from a unique id in C++,
all-gathers host buffers (the expansion's error headers) and device buffers on a stream (the
per-wave records).  One GPU here, so world = 1; the sharded expansion with world > 1 is covered by
the in-process exchange tests (test_gpu_expand.py) and runs over this communicator in bench.py's
shard mode."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_allgather(gpu_available):
    import pmvs_amd as P
    uid = P.RcclExchange.unique_id()
    assert len(uid) == 128
    ex = P.RcclExchange(0, 1, uid, device=0)
    data = bytes(range(200))
    assert ex.allgather(data) == data
    ex.close()


def test_rccl_device_allgather_and_scene_attach(gpu_available):
    import torch
    import pmvs_amd as P
    ex = P.RcclExchange(0, 1, P.RcclExchange.unique_id(), device=0)
    src = torch.arange(1000, dtype=torch.int32, device="cuda:0")
    dst = torch.zeros_like(src)
    s = torch.cuda.current_stream()
    f = ex.lib.pmvs_rccl_allgather_device
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    f.restype = C.c_int
    assert f(ex.handle, src.data_ptr(), src.numel() * 4, dst.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    inp, _ = P.synth_scene(3, 64, 48, level=1)
    sc = P.Scene(inp)
    ex.attach(sc)  # world 1: sharding stays off, the call is accepted
    sc.close()
    ex.close()
