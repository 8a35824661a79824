"""The C-ABI collective (csrc/comm.hip; SURVEY.md §8 b insr_comm_init / insr_allreduce_sum)
on the GPU box: a one-rank RCCL communicator (the box has one GPU) -- unique id, init,
in-place sum all-reduce of a flat gradient buffer on the torch stream (identity for one
rank), destroy.  The multi-rank reduction itself is the same RCCL call torch.distributed
makes in BaseModel._dp_sync (covered by tests/test_dp_gloo.py and test_gpu_dp.py)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_comm_single_rank_allreduce():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    nat = base._native
    lib = nat.load()
    assert lib.insr_comm_available() == 1
    idb = ctypes.create_string_buffer(lib.insr_comm_id_bytes())
    assert lib.insr_comm_unique_id(idb) == 0
    comm = ctypes.c_void_p()
    assert lib.insr_comm_init(ctypes.byref(comm), 0, 1, idb) == 0
    buf = torch.randn(533 * 256, device="cuda")  # ~ the fluid gradient + loss message
    ref = buf.clone()
    assert lib.insr_comm_allreduce_sum(comm, nat.ptr(buf), buf.numel(), nat.stream_of(buf.device)) == 0
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    assert lib.insr_comm_allreduce_sum(comm, None, 0, nat.stream_of(buf.device)) == 0
    assert lib.insr_comm_destroy(comm) == 0
