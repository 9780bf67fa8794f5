"""The N>1 exchange's host logic on the CPU: the file rendezvous of the RCCL
unique id between real processes (the RCCL calls themselves need a GPU:
tests/test_gpu_comm.py), and the ABI's communicator entry points."""
import multiprocessing as mp
import os
import uuid

import pytest

from ldpc_amd import comm


def _rank(rank, world, key, q):
    uid = comm.file_rendezvous(rank, world, lambda: bytes(range(128)) if rank == 0 else None, key=key,
                               timeout=60)
    q.put((rank, uid))


def test_file_rendezvous_two_processes():
    key = uuid.uuid4().hex
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    # rank 1 starts first: it must wait for rank 0's file, never read a partial one
    ps = [ctx.Process(target=_rank, args=(r, 2, key, q)) for r in (1, 0)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert got[0] == got[1] == bytes(range(128))
    os.unlink(comm.rendezvous_path(key))


def test_file_rendezvous_times_out():
    with pytest.raises(TimeoutError):
        comm.file_rendezvous(1, 2, None, key=uuid.uuid4().hex, timeout=0.3)


def test_rendezvous_key_is_per_launch(monkeypatch):
    monkeypatch.setenv("MASTER_PORT", "29511")
    p = comm.rendezvous_path()
    assert f"_{os.getppid()}_29511" in p
