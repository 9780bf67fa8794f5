"""Multi-GPU counter exchange: RCCL behind the C ABI (no PyTorch).

One process per GPU, started by torch.distributed.run or by bench.py's own
launcher (bench.py --gpus N with no launcher around it); either sets RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_PORT, bench.py's launcher also LDPC_RDV_KEY.  Frames
shard by global index (montecarlo.shard), so the one collective is the
all-reduce of the int64 counter matrix -- the reference's parent-side sum of
its workers' per-block results (python_ldpc_app/main.py:149-175).

Rendezvous: rank 0 asks RCCL for a 128-byte unique id (ldpc_comm_unique_id)
and publishes it in a file; the other ranks poll for it.  The file is named
by a key every rank of ONE launch attempt shares and no other attempt does:
LDPC_RDV_KEY when the launcher sets one (bench.py: a fresh uuid per launch),
else the launcher's pid (os.getppid()) + MASTER_PORT + torchelastic's run id
and restart count (an elastic restart keeps the agent pid and the port), so a
stale file of an earlier launch or attempt is never read.  Single node only
(--nnodes=1, as the driver runs it).
"""
import ctypes
import os
import tempfile
import time

import numpy as np

from . import _lib
from ._lib import LDPC_F_DEVICE_PTRS, check

ID_BYTES = 128
DT = {np.dtype(np.int64): 0, np.dtype(np.float64): 1}
OPS = {"sum": 0, "max": 1}


def rendezvous_key():
    k = os.environ.get("LDPC_RDV_KEY")
    if k:
        return k
    e = os.environ
    return "_".join([str(os.getppid()), e.get("MASTER_PORT", "0"), e.get("TORCHELASTIC_RUN_ID", "none"),
                     e.get("TORCHELASTIC_RESTART_COUNT", "0")])


def rendezvous_path(key=None):
    key = "".join(ch if ch.isalnum() or ch in "_-" else "-" for ch in (key or rendezvous_key()))
    return os.path.join(tempfile.gettempdir(), f"ldpc_rccl_{key}.id")


def file_rendezvous(rank, world, make_id, key=None, timeout=300.0):
    """Rank 0 publishes make_id() (bytes) in a file, every rank returns it."""
    path = rendezvous_path(key)
    if rank == 0:
        uid = bytes(make_id())
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as fh:
            fh.write(uid)
        os.replace(tmp, path)  # atomic: readers see all bytes or nothing
        return uid
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as fh:
                uid = fh.read()
            if len(uid) == ID_BYTES:
                return uid
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}/{world}: no RCCL id at {path} after {timeout:.0f} s")
        time.sleep(0.05)


def rccl_unique_id():
    buf = (ctypes.c_uint8 * ID_BYTES)()
    check("ldpc_comm_unique_id", _lib.gpu().ldpc_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """An RCCL communicator of `world` ranks, this process = `rank` on GPU `device`."""

    def __init__(self, rank, world, device, uid):
        self.rank, self.world, self.device = int(rank), int(world), int(device)
        idbuf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        check("ldpc_comm_init", _lib.gpu().ldpc_comm_init(idbuf, self.rank, self.world, self.device,
                                                          ctypes.byref(h)))
        self._h = h
        self._pid = os.getpid()

    @classmethod
    def from_env(cls, device=None):
        """RANK / WORLD_SIZE / LOCAL_RANK from the launcher; file rendezvous."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
        uid = file_rendezvous(rank, world, rccl_unique_id)
        c = cls(rank, world, dev, uid)
        c.barrier()
        if rank == 0:  # every rank has read the id
            try:
                os.unlink(rendezvous_path())
            except OSError:
                pass
        return c

    def allreduce(self, arr, op="sum"):
        """In-place-style all-reduce of a host int64/float64 array; returns the result."""
        a = np.ascontiguousarray(np.array(arr, copy=True))
        if a.dtype not in DT:
            raise TypeError(f"allreduce: dtype {a.dtype} (int64 or float64 only)")
        check("ldpc_comm_allreduce", _lib.gpu().ldpc_comm_allreduce(
            self._h, a.ctypes.data, a.size, DT[a.dtype], OPS[op], 0, None))
        return a

    def allreduce_device(self, ptr, count, dtype=np.int64, op="sum", stream=None):
        """Device buffer (anything with data_ptr() or an int address), async on `stream`."""
        addr = int(ptr.data_ptr()) if hasattr(ptr, "data_ptr") else int(ptr)
        check("ldpc_comm_allreduce", _lib.gpu().ldpc_comm_allreduce(
            self._h, ctypes.c_void_p(addr), int(count), DT[np.dtype(dtype)], OPS[op], LDPC_F_DEVICE_PTRS,
            ctypes.c_void_p(int(stream)) if stream else None))

    def barrier(self):
        check("ldpc_comm_barrier", _lib.gpu().ldpc_comm_barrier(self._h))

    def ranks_seen(self):
        """How many ranks answer on this communicator: an RCCL sum of one per
        rank (what ldpc_comm_barrier checks against world)."""
        return int(self.allreduce(np.ones(1, np.int64))[0])

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None and getattr(self, "_pid", None) == os.getpid():
            _lib._lib.ldpc_comm_destroy(h)
        self._h = None

    def __del__(self):
        self.close()


def device_synchronize(device):
    check("ldpc_device_synchronize", _lib.gpu().ldpc_device_synchronize(int(device)))
