"""Python handles over the C ABI: the graph on a GPU and a decoder workspace.

``Graph``   wraps ldpc_graph_create (H_std uploaded once per device, cached by
            content and process so repeated SPA_Decoder constructions --
            main.py:221 builds one per SNR point, main.py:78 one per frame --
            do not re-upload, and a forked worker never gets its parent's
            device handle).
``Decoder`` wraps ldpc_decoder_create / ldpc_decode_f64 / ldpc_mc_run.
Every call here goes through _lib.gpu() (fork check, _lib's docstring); a
handle is only released by the process that created it.
"""
import ctypes
import hashlib
import os
import threading

import numpy as np
from scipy import sparse

from . import _lib
from ._lib import (LDPC_EINVAL, LDPC_ERANGE, LDPC_F_DEVICE_PTRS, LDPC_F_NLLR, LDPC_F_PHYS_HBM, LDPC_F_SPLIT,
                   LDPC_F_STATIC, LDPC_MC_NCOUNT, LdpcError, as_i32, check)


def _csr_arrays(H):
    H = sparse.csr_matrix(H)
    if not H.has_sorted_indices:
        H = H.sorted_indices()
    return H.shape[0], H.shape[1], as_i32(H.indptr), as_i32(H.indices)


def validate_csr(m, n, indptr, indices):
    """ldpc_graph_create's argument checks (csrc/ldpc_api.cpp), HIP-free, so a
    bad H fails where it is handed over (SPA_Decoder.__init__ in the parent
    process, as the reference's constructor would) rather than on the first
    decode() inside a forked worker.  Raises LdpcError with the C codes."""
    fn = "ldpc_graph_create"
    if m <= 0 or n <= 0 or m > n:
        raise LdpcError(fn, LDPC_EINVAL, f"bad shape m={m} n={n}")
    indptr = np.asarray(indptr)
    indices = np.asarray(indices)
    if len(indptr) != m + 1 or indptr[0] != 0:
        raise LdpcError(fn, LDPC_EINVAL, "row_ptr[0] != 0")
    nnz = int(indptr[-1])
    lim = (2 ** 31 - 1) // 64  # within-tile offsets are 32-bit: e * 64 must fit
    if nnz <= 0 or nnz > lim or n > lim:
        raise LdpcError(fn, LDPC_ERANGE, f"nnz={nnz} outside 32-bit tile indexing")
    d = np.diff(indptr)
    if (d < 0).any():
        raise LdpcError(fn, LDPC_EINVAL, f"row_ptr not monotone at {int(np.argmax(d < 0))}")
    if len(indices) < nnz or (indices[:nnz] < 0).any() or (indices[:nnz] >= n).any():
        raise LdpcError(fn, LDPC_EINVAL, "column out of range")
    c = indices[:nnz].astype(np.int64)
    step = np.diff(c)
    same_row = np.ones(max(nnz - 1, 0), bool)
    same_row[(indptr[1:-1][(indptr[1:-1] > 0) & (indptr[1:-1] < nnz)] - 1)] = False
    bad = (step <= 0) & same_row
    if bad.any():
        r = int(np.searchsorted(indptr, int(np.argmax(bad)) + 1, side="right") - 1)
        raise LdpcError(fn, LDPC_EINVAL, f"row {r} columns not strictly ascending "
                                         "(the reference's check_to_var order is required)")


class Graph:
    """H_std (CSR, ascending columns) resident on one GPU."""

    _cache = {}
    _cache_lock = threading.Lock()

    def __init__(self, H, device=-1):
        m, n, indptr, indices = _csr_arrays(H)
        self.m, self.n, self.k = m, n, n - m
        self.indptr, self.indices = indptr, indices
        self.nnz = int(indptr[-1])
        h = ctypes.c_void_p()
        check("ldpc_graph_create", _lib.gpu().ldpc_graph_create(
            m, n, _lib.i32p(indptr), _lib.i32p(indices), int(device), ctypes.byref(h)))
        self._h = h
        self._pid = os.getpid()
        mr, mc = ctypes.c_int32(), ctypes.c_int32()
        check("ldpc_graph_info", _lib.gpu().ldpc_graph_info(h, None, None, None, ctypes.byref(mr), ctypes.byref(mc)))
        self.max_row_deg, self.max_col_deg = mr.value, mc.value

    @property
    def handle(self):
        return self._h

    @classmethod
    def cached(cls, H, device=-1):
        m, n, indptr, indices = _csr_arrays(H)
        key = (os.getpid(), m, n, int(device), hashlib.sha1(indptr.tobytes() + indices.tobytes()).hexdigest())
        with cls._cache_lock:
            g = cls._cache.get(key)
            if g is None:
                g = cls(sparse.csr_matrix((np.ones(len(indices), np.int32), indices, indptr), shape=(m, n)), device)
                cls._cache[key] = g
        return g

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None and getattr(self, "_pid", None) == os.getpid():
            _lib._lib.ldpc_graph_destroy(h)
        self._h = None


def phys_decode(graph, llr, max_iter, post=False, hbm=False):
    """Physical-mode decode of [B, n] LLRs on a sparse graph (H[:, perm]).

    State in LDS when a frame fits, else in HBM (hbm=True forces HBM)."""
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, dtype=np.float64)))
    B, n = llr.shape
    if n != graph.n:
        raise ValueError(f"llr must be [batch, {graph.n}]")
    z = np.empty((B, n), np.uint8)
    conv = np.empty(B, np.int32)
    status = np.empty(B, np.int32)
    iters = np.empty(B, np.int32)
    Lp = np.empty((B, n), np.float32) if post else None
    check("ldpc_phys_decode", _lib.gpu().ldpc_phys_decode(
        graph.handle, B, _lib.ptr(llr), int(max_iter), LDPC_F_PHYS_HBM if hbm else 0, _lib.ptr(z), _lib.ptr(conv),
        _lib.ptr(status),
        _lib.ptr(iters), _lib.ptr(Lp), None))
    return DecodeResult(z=z, conv=conv, status=status, iters=iters, post=Lp)


class DecodeResult(dict):
    __getattr__ = dict.__getitem__


class Decoder:
    """Device workspace for chunks of up to `max_frames` frames."""

    def __init__(self, graph, max_frames=4096):
        self.graph = graph
        h = ctypes.c_void_p()
        check("ldpc_decoder_create", _lib.gpu().ldpc_decoder_create(graph.handle, int(max_frames), ctypes.byref(h)))
        self._h = h
        self._pid = os.getpid()
        self.capacity = int(_lib.gpu().ldpc_decoder_capacity(h))

    @staticmethod
    def workspace_bytes(graph, max_frames):
        return int(_lib.gpu().ldpc_decoder_bytes(graph.handle, int(max_frames)))

    # HBM the Monte-Carlo drivers let one decoder take (of 288 GB per MI355X);
    # LDPC_HBM_BUDGET_GB overrides
    HBM_BUDGET = 160e9

    @classmethod
    def fit_slots(cls, graph, frames, budget=None):
        """Slots (resident frames, a multiple of 64) for a workspace of at most
        `budget` bytes, and no more than `frames`: fp64 messages are 8 B per
        edge per frame, 5.3 MB for wimax_2304_0.5, so its 65,536-frame batch
        (348 GB) streams through ~30k slots instead."""
        if budget is None:
            budget = float(os.environ.get("LDPC_HBM_BUDGET_GB", cls.HBM_BUDGET / 1e9)) * 1e9
        # workspace = fixed (rare-row scratch, graph-sized buffers) + per-frame state
        a, b = 64 * 64, 2 * 64 * 64
        wa, wb = cls.workspace_bytes(graph, a), cls.workspace_bytes(graph, b)
        per = (wb - wa) / (b - a)
        fixed = wa - per * a
        fit = max(64, int((budget - fixed) // per) // 64 * 64)
        return max(1, min(int(frames), fit))

    def decode(self, llr, max_iter, nllr=False, post=False, hist=False, msgs=False, split=False):
        """Decode [B, n] channel LLRs (H_std column order).  Returns numpy arrays.

        split=True forces the per-iteration CN/VN launches where the
        tile-resident decoder would run (same results; A/B and tests)."""
        g = self.graph
        llr = np.ascontiguousarray(np.asarray(llr, dtype=np.float64))
        if llr.ndim == 1:
            llr = llr[None, :]
        if llr.ndim != 2 or llr.shape[1] != g.n:
            raise ValueError(f"llr must be [batch, {g.n}], got {llr.shape}")
        B = llr.shape[0]
        T = int(max_iter)
        z = np.empty((B, g.n), np.uint8)
        conv = np.empty(B, np.int32)
        status = np.empty(B, np.int32)
        iters = np.empty(B, np.int32)
        nl = np.zeros(B, np.float64) if nllr else None
        Lp = np.empty((B, g.n), np.float64) if post else None
        hi = np.empty((B, T), np.float64) if (hist and nllr) else None
        E = np.empty((B, g.nnz), np.float64) if msgs else None
        flags = (LDPC_F_NLLR if nllr else 0) | (LDPC_F_SPLIT if split else 0)
        check("ldpc_decode_f64", _lib.gpu().ldpc_decode_f64(
            self._h, B, _lib.ptr(llr), T, flags, _lib.ptr(z), _lib.ptr(conv), _lib.ptr(status),
            _lib.ptr(Lp), _lib.ptr(nl), _lib.ptr(hi), _lib.ptr(iters), _lib.ptr(E), None))
        return DecodeResult(z=z, conv=conv, status=status, iters=iters, nllr=nl, post=Lp, hist=hi, msgs=E)

    def decode_device(self, llr, max_iter, z=None, conv=None, status=None, post=None, nllr=None, hist=None,
                      iters=None, split=False, stream=None):
        """LDPC_F_DEVICE_PTRS: every buffer is device memory (anything with a
        data_ptr(), e.g. a torch CUDA tensor: llr [B, n] f64, z [B, n] u8,
        conv / status / iters [B] i32, post [B, n] f64, nllr [B] f64, hist
        [B, max_iter] f64), and the call is asynchronous on `stream` (a
        hipStream_t handle as int; None = the null stream) unless nllr or hist
        is requested.  Same results as decode()."""
        def dp(t):
            return None if t is None else ctypes.c_void_p(int(t.data_ptr()))
        B, n = int(llr.shape[0]), int(llr.shape[1])
        if n != self.graph.n:
            raise ValueError(f"llr must be [batch, {self.graph.n}]")
        flags = LDPC_F_DEVICE_PTRS | (LDPC_F_NLLR if (nllr is not None or hist is not None) else 0) | \
            (LDPC_F_SPLIT if split else 0)
        check("ldpc_decode_f64", _lib.gpu().ldpc_decode_f64(
            self._h, B, dp(llr), int(max_iter), flags, dp(z), dp(conv), dp(status), dp(post), dp(nllr), dp(hist),
            dp(iters), None, ctypes.c_void_p(int(stream)) if stream else None))

    def generate(self, seed, snr_point, sigma, frame0, count, test_zero=False):
        """On-device synthetic frames (u bits, channel LLRs) copied back for testing.
        test_zero: the frame source's test-only erasures (LDPC_F_TEST_ZERO)."""
        g = self.graph
        u = np.empty((count, g.k), np.uint8)
        llr = np.empty((count, g.n), np.float64)
        check("ldpc_generate_frames", _lib.gpu().ldpc_generate_frames(
            self._h, int(seed), int(snr_point), float(sigma), int(frame0), int(count),
            _lib.LDPC_F_TEST_ZERO if test_zero else 0, _lib.ptr(u), _lib.ptr(llr), None))
        return u, llr

    def mc_run(self, seed, sigmas, frames_per_point, frame0, max_iter, nllr=False, static=False, split=False,
               test_zero=False):
        """Generate + decode + count on the GPU; returns int64 [n_points, 7] counters.

        Default schedule streams frames through the decoder's slots (a slot is
        refilled as soon as its frame stops); static=True decodes chunks of
        capacity frames to completion.  Same frames, identical counters.
        test_zero: the frame source's test-only erasures (LDPC_F_TEST_ZERO)."""
        sig = np.ascontiguousarray(np.asarray(sigmas, dtype=np.float64))
        out = np.zeros((len(sig), LDPC_MC_NCOUNT), np.int64)
        flags = (LDPC_F_NLLR if nllr else 0) | (LDPC_F_STATIC if static else 0) | (LDPC_F_SPLIT if split else 0) | \
            (_lib.LDPC_F_TEST_ZERO if test_zero else 0)
        check("ldpc_mc_run", _lib.gpu().ldpc_mc_run(
            self._h, int(seed), len(sig), sig.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
            int(frames_per_point), int(frame0), int(max_iter), flags,
            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None))
        return out

    def frame_order(self, seed, snr_point, sigma, frame0, count):
        """The streaming schedule's supply order of a point (ldpc_frame_order):
        local frame indices by descending syndrome weight of their channel hard
        decisions, ties in index order."""
        out = np.empty(int(count), np.int32)
        check("ldpc_frame_order", _lib.gpu().ldpc_frame_order(
            self._h, int(seed), int(snr_point), float(sigma), int(frame0), int(count), _lib.ptr(out), None))
        return out

    def phys_mc_run(self, phys_graph, seed, sigmas, frames_per_point, frame0, max_iter, hbm=False):
        """Physical mode (§8 f4): same on-device frames, decoded on the sparse graph.

        This decoder's graph is the code's H_std (frame source) or, for an IRA
        code, phys_graph itself.  hbm=True forces the HBM-resident tile path."""
        sig = np.ascontiguousarray(np.asarray(sigmas, dtype=np.float64))
        out = np.zeros((len(sig), LDPC_MC_NCOUNT), np.int64)
        check("ldpc_phys_mc_run", _lib.gpu().ldpc_phys_mc_run(
            self._h, phys_graph.handle, int(seed), len(sig), sig.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
            int(frames_per_point), int(frame0), int(max_iter), LDPC_F_PHYS_HBM if hbm else 0,
            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None))
        return out

    KINDS = ("cn", "vn", "generate", "count", "phys", "phys_cn", "phys_vn", "tile", "cn_edge", "vn_edge",
             "vn_cols")

    def profile(self, enable=True):
        check("ldpc_profile_enable", _lib.gpu().ldpc_profile_enable(self._h, 1 if enable else 0))

    def profile_read(self):
        """{kind: (total_ms, launches)} of this decoder's launches since the last read."""
        ms = (ctypes.c_double * len(self.KINDS))()
        n = (ctypes.c_int64 * len(self.KINDS))()
        check("ldpc_profile_read", _lib.gpu().ldpc_profile_read(self._h, ms, n))
        return {k: (ms[i], n[i]) for i, k in enumerate(self.KINDS)}

    def rare_rows(self):
        """(rows queued to cn_rare_kernel, rare rows the tile decoders took in-kernel)
        since the last call (ldpc_rare_rows_read)."""
        out = (ctypes.c_int64 * 2)()
        check("ldpc_rare_rows_read", _lib.gpu().ldpc_rare_rows_read(self._h, out))
        return int(out[0]), int(out[1])

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None and getattr(self, "_pid", None) == os.getpid():
            _lib._lib.ldpc_decoder_destroy(h)
        self._h = None

    def __del__(self):
        self.close()
