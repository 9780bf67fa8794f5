"""RCCL behind the C ABI (ldpc_comm_*), world size 1 on the GPU box (the
driver's 8-GPU node runs bench.py --gpus N through the same calls)."""
import numpy as np
import pytest

from ldpc_amd import comm

pytestmark = pytest.mark.gpu


def test_rccl_world1_allreduce_and_barrier(gpu_available):
    uid = comm.rccl_unique_id()
    assert len(uid) == comm.ID_BYTES
    c = comm.Comm(0, 1, 0, uid)
    try:
        ctr = np.arange(14, dtype=np.int64).reshape(2, 7) * 1_000_003
        out = c.allreduce(ctr)
        assert out.dtype == np.int64 and np.array_equal(out, ctr)  # sum over one rank
        assert float(c.allreduce(np.array([2.5]), op="max")[0]) == 2.5
        c.barrier()
        comm.device_synchronize(0)
    finally:
        c.close()


def test_rccl_rejects_bad_arguments(gpu_available):
    from ldpc_amd import LdpcError
    with pytest.raises(LdpcError):
        comm.Comm(1, 1, 0, bytes(128))  # rank outside world
    c = comm.Comm(0, 1, 0, comm.rccl_unique_id())
    try:
        with pytest.raises(TypeError):
            c.allreduce(np.zeros(3, np.int32))
    finally:
        c.close()
