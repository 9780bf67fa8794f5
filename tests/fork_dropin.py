"""main.py's multi-process pattern against the drop-in decoder (GPU).

python_ldpc_app/main.py:221 builds an SPA_Decoder in the parent for every SNR
point and then (``--threads P > 1``, main.py:248-256) forks a
ProcessPoolExecutor whose workers each build their own decoder per block
(process_block, main.py:78) and decode one frame (main.py:123-124).
adaptive.py:227-282 does the same.  run() replays that on the golden frames
of tests/golden/w576_T5.npz (reference outputs) and returns the mismatches.

Must start in a process that has not started HIP (tests/test_gpu_00_fork.py
runs first in the GPU session, or runs this file as a script).
"""
import multiprocessing as mp
import os
import sys
from concurrent.futures import ProcessPoolExecutor, as_completed

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "ldpc-simulator_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


class _Buffer:
    """The two DataBuffer attributes decode() uses (data_buffer.py:16-45)."""

    def __init__(self, ch):
        self._channel_data = [float(x) for x in ch]
        self._decoded_data = None


class Edd:
    """The three attributes SPA_Decoder reads (spa_decoder.py:28-31); picklable,
    as main.py ships its EncoderDecoderData to the workers by pickle."""


def _settings(T, nllr):
    from ldpc_amd.settings import Settings
    s = Settings()
    s.set_max_iterations(int(T))
    s.set_normalized_llr_calculate(bool(nllr))
    return s


def process_block(i, edd, settings, ch):
    """process_block (main.py:43-146) reduced to the decoder's part."""
    import ldpc_amd
    decoder = ldpc_amd.SPA_Decoder(edd, settings)  # main.py:78 -- one per block, in the worker
    db = _Buffer(ch)
    res = decoder.decode(db)  # main.py:124
    return i, os.getpid(), np.asarray(db._decoded_data, np.uint8), decoder.convergence_iteration, res.name


def run(workers=2, frames=16):
    import ldpc_amd
    from ldpc_amd import _lib
    from conftest import hstd_for, load_golden

    g = load_golden("w576_T5")
    H = hstd_for(str(g["code"]))

    edd = Edd()
    edd._h_sparse_cached, edd._m, edd._n = H, H.shape[0], H.shape[1]
    settings = _settings(int(g["T"]), bool(g["nllr_on"]))
    assert not _lib.hip_started_here(), "run() must start in a process without HIP"
    parent = ldpc_amd.SPA_Decoder(edd, settings)  # main.py:221, before the fork
    assert not _lib.hip_started_here(), "SPA_Decoder.__init__ started the HIP runtime"
    bad, pids = [], set()
    with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("fork")) as ex:
        futs = [ex.submit(process_block, i, edd, settings, g["ch"][i]) for i in range(frames)]
        for fu in as_completed(futs):
            i, pid, z, conv, res = fu.result()
            pids.add(pid)
            if not (np.array_equal(z, g["z"][i]) and conv == int(g["conv"][i])
                    and (res == "OK") == bool(g["ok"][i])):
                bad.append(i)
    # the parent's own decoder still works afterwards (it starts HIP here)
    db = _Buffer(g["ch"][0])
    parent.decode(db)
    if not np.array_equal(np.asarray(db._decoded_data, np.uint8), g["z"][0]):
        bad.append("parent")
    return bad, pids


def run_poisoned():
    """A child forked AFTER the parent started HIP must refuse, not hang."""
    import ldpc_amd
    from ldpc_amd import _lib
    ldpc_amd.device_count()
    assert _lib.hip_started_here()
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def child(q):
        try:
            ldpc_amd.device_count()
            q.put("no error")
        except ldpc_amd.LdpcError as e:
            q.put("refused" if e.code == _lib.LDPC_EFORK else f"other: {e}")

    p = ctx.Process(target=child, args=(q,))
    p.start()
    out = q.get(timeout=60)
    p.join(60)
    return out


if __name__ == "__main__":
    bad, pids = run()
    print(f"mismatches={bad} worker_pids={len(pids)}")
    print(f"poisoned_child={run_poisoned()}")
    sys.exit(1 if bad else 0)
