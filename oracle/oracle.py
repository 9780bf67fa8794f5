"""Python access to the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package (ldpc-simulator_amd/ldpc_amd) never does.

  spa_decode(...)       -> oracle/spa_oracle.c   (restates spa_decoder.py:63-280)
  generate_frames(...)  -> oracle/channel_oracle.c (restates our device frame source)
  main_counters(...)    -> numpy restatement of main.py:130-138,154-172,346-369

Parity status: pinned.  tests/test_oracle_golden.py checks spa_decode against
every golden vector produced by the reference itself (tests/golden/gen_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_spa.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(LIB):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        vp, i32, i64, u64, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
        L.oracle_spa_decode_batch.restype = ctypes.c_int
        L.oracle_spa_decode_batch.argtypes = [i32, i32, vp, vp, i32, vp, i32, i32, i32,
                                              vp, vp, vp, vp, vp, vp, vp]
        L.oracle_generate_frames.restype = ctypes.c_int
        L.oracle_generate_frames.argtypes = [i32, i32, vp, vp, u64, i32, dbl, i64, i32, vp, vp, vp]
        L.oracle_ira_generate_frames.restype = ctypes.c_int
        L.oracle_ira_generate_frames.argtypes = [i32, i32, vp, vp, u64, i32, dbl, i64, i32, vp, vp, vp]
        L.oracle_philox4x32_10.restype = None
        L.oracle_philox4x32_10.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_max_threads.restype = ctypes.c_int
        L.oracle_phys_decode.restype = ctypes.c_int
        L.oracle_phys_decode.argtypes = [i32, i32, vp, vp, i32, vp, i32, vp, vp, vp, vp]
        L.oracle_np_tanh.restype = dbl
        L.oracle_np_tanh.argtypes = [dbl]
        L.oracle_set_tanh_nudge.restype = None
        L.oracle_set_tanh_nudge.argtypes = [i32]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def _csr(H):
    from scipy import sparse
    H = sparse.csr_matrix(H)
    return (H.shape[0], H.shape[1], np.ascontiguousarray(H.indptr, dtype=np.int32),
            np.ascontiguousarray(H.indices, dtype=np.int32))


def spa_decode(H_std, llr, max_iter, nllr=False, want_L=True, want_E=False, threads=0):
    """Decode [B, n] LLRs on the CPU exactly as spa_decoder.py does."""
    m, n, indptr, indices = _csr(H_std)
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, dtype=np.float64)))
    B = llr.shape[0]
    nnz = int(indptr[-1])
    z = np.empty((B, n), np.uint8)
    conv = np.empty(B, np.int32)
    status = np.empty(B, np.int32)
    iters = np.empty(B, np.int32)
    nl = np.zeros(B, np.float64)
    L = np.empty((B, n), np.float64) if want_L else None
    E = np.empty((B, nnz), np.float64) if want_E else None
    rc = lib().oracle_spa_decode_batch(m, n, _p(indptr), _p(indices), B, _p(llr), int(max_iter),
                                       1 if nllr else 0, int(threads), _p(z), _p(conv), _p(status),
                                       _p(L), _p(E), _p(nl), _p(iters))
    if rc != 0:
        raise ValueError("oracle_spa_decode_batch rejected its arguments")
    return dict(z=z, conv=conv, status=status, iters=iters, nllr=nl, post=L, msgs=E)


def conditioning_slack(H_std, llr, max_iter, nllr=False, factor=4.0):
    """Elementwise slack for L and E: `factor` x how far ONE ulp of tanh moves them.

    Returns (slack_L [B,n], slack_E [B,nnz]).  Zero (to rounding) for well
    conditioned frames; large only for frames saturated at the +-CL clip.
    """
    base = spa_decode(H_std, llr, max_iter, nllr=nllr, want_E=True)
    lib().oracle_set_tanh_nudge(1)
    try:
        pert = spa_decode(H_std, llr, max_iter, nllr=nllr, want_E=True)
    finally:
        lib().oracle_set_tanh_nudge(0)
    return factor * np.abs(pert["post"] - base["post"]), factor * np.abs(pert["msgs"] - base["msgs"])


def phys_decode(H_phys, llr, max_iter):
    """CPU restatement of the physical mode (our design, oracle/phys_oracle.c)."""
    m, n, indptr, indices = _csr(H_phys)
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, dtype=np.float64)))
    B = llr.shape[0]
    z = np.empty((B, n), np.uint8)
    conv = np.empty(B, np.int32)
    iters = np.empty(B, np.int32)
    post = np.empty((B, n), np.float32)
    if lib().oracle_phys_decode(m, n, _p(indptr), _p(indices), B, _p(llr), int(max_iter),
                                _p(z), _p(conv), _p(iters), _p(post)) != 0:
        raise ValueError("oracle_phys_decode rejected its arguments")
    return dict(z=z, conv=conv, status=(conv < 0).astype(np.int32), iters=iters, post=post)


def np_tanh(x):
    """The oracle's restatement of numpy's float64 tanh (elementwise)."""
    f = lib().oracle_np_tanh
    return np.array([f(float(v)) for v in np.asarray(x, dtype=np.float64).ravel()]).reshape(np.shape(x))


def generate_frames(H_std, seed, snr_point, sigma, frame0, count, ira=False):
    """Frames of the on-device source: H_std = [A | I] (c = [u, A u]) or, with
    ira=True, an IRA H = [H_info | staircase] (c = [u, accumulated parities])."""
    m, n, indptr, indices = _csr(H_std)
    k = n - m
    u = np.empty((count, k), np.uint8)
    c = np.empty((count, n), np.uint8)
    llr = np.empty((count, n), np.float64)
    fn = lib().oracle_ira_generate_frames if ira else lib().oracle_generate_frames
    rc = fn(m, n, _p(indptr), _p(indices), int(seed), int(snr_point), float(sigma),
            int(frame0), int(count), _p(u), _p(c), _p(llr))
    if rc != 0:
        raise ValueError("oracle_generate_frames rejected its arguments")
    return u, c, llr


def philox(ctr, key):
    c = np.ascontiguousarray(np.asarray(ctr, dtype=np.uint32))
    lib().oracle_philox4x32_10(c.ctypes.data, int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF)
    return c


def main_counters(u, z, status, conv, nllr_cnt=None, iters=None):
    """Per-SNR counter vector, main.py:130-138 (BER only over failed frames) + :154-172."""
    u = np.asarray(u, dtype=np.uint8)
    k = u.shape[1]
    ok = np.asarray(status) == 0
    dec = (np.asarray(z)[:, :k] ^ 1).astype(np.uint8)
    err = np.where(ok, 0, (dec != u).sum(axis=1))
    conv = np.asarray(conv)
    out = np.zeros(7, np.int64)
    out[0] = len(ok)
    out[1] = int((~ok).sum())
    out[2] = int(err.sum())
    out[3] = int(conv[conv >= 0].sum())
    out[4] = int((conv >= 0).sum())
    out[5] = 0 if nllr_cnt is None else int(np.asarray(nllr_cnt).sum())
    out[6] = 0 if iters is None else int(np.asarray(iters).sum())
    return out


def sigma_for_snr(snr_db, speed=1.0):
    """channel.py:113 (mode 1): 1/sqrt(2*speed*10^(snr/10))."""
    import math
    return 1.0 / math.sqrt(2.0 * speed * (10.0 ** (snr_db * 0.1)))
