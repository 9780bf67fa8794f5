"""Code construction: ALIST H -> standard form H_std = [A | I_m] (graph provider).

Mirrors python_ldpc_app/encoder_decoder_data.py:EncoderDecoderData (lines
186-267) for the attributes the decoder path reads: _h, _n, _m,
_k, _rate, _h_std, _permutation, _h_sparse_cached, _g_transpose.  The GF(2)
elimination runs natively (ldpc_hstd_build, csrc/hstd_builder.cpp) instead of
the reference's pure-Python loop (:13-183); the result is the same RREF and
permutation (pinned by sha256 against the reference; the per-code data --
ALIST-derived H, H_std / permutation fingerprints -- ships with the package in
ldpc_amd/codes/, written by tests/golden/gen_golden.py from the reference).
Matrices are scipy CSR (the reference wraps the same in SparseMatrix).
"""
import ctypes
import hashlib
import os

import numpy as np
from scipy import sparse

from . import _lib
from ._lib import as_i32, check
from .alist import read_parity_check_matrix

HERE = os.path.dirname(os.path.abspath(__file__))
CODES_DIR = os.path.join(HERE, "codes")  # ALIST-derived H + fingerprints of the reference's codes


def build_standard_form(H):
    """GF(2) Gauss-Jordan via the native builder.

    Returns (H_std CSR [rank x n], permutation list).  encoder_decoder_data.py:269-317.
    """
    H = sparse.csr_matrix(H)
    m, n = H.shape
    indptr, indices = as_i32(H.indptr), as_i32(H.indices)
    L = _lib.lib()
    h = ctypes.c_void_p()
    check("ldpc_hstd_build", L.ldpc_hstd_build(m, n, _lib.i32p(indptr), _lib.i32p(indices), ctypes.byref(h)))
    try:
        ms, nn, nnz = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        rp, ci, pm = (ctypes.POINTER(ctypes.c_int32)(), ctypes.POINTER(ctypes.c_int32)(),
                      ctypes.POINTER(ctypes.c_int32)())
        check("ldpc_hstd_get", L.ldpc_hstd_get(h, ctypes.byref(ms), ctypes.byref(nn), ctypes.byref(nnz),
                                               ctypes.byref(rp), ctypes.byref(ci), ctypes.byref(pm)))
        rank = ms.value
        row_ptr = np.ctypeslib.as_array(rp, shape=(rank + 1,)).copy()
        col_idx = np.ctypeslib.as_array(ci, shape=(max(nnz.value, 1),))[:nnz.value].copy()
        perm = np.ctypeslib.as_array(pm, shape=(n,)).copy()
    finally:
        L.ldpc_hstd_free(h)
    Hs = sparse.csr_matrix((np.ones(len(col_idx), np.int32), col_idx, row_ptr), shape=(rank, n))
    return Hs, perm.tolist()


def csr_fingerprint(H):
    """sha256(int32-LE indptr || int32-LE indices) -- SURVEY.md §8c convention."""
    H = sparse.csr_matrix(H)
    return hashlib.sha256(as_i32(H.indptr).astype("<i4").tobytes() + as_i32(H.indices).astype("<i4").tobytes()).hexdigest()


class EncoderDecoderData:
    """Parity-check data for one code.  `source` is an ALIST path or a matrix H."""

    def __init__(self, source):
        if isinstance(source, (str, os.PathLike)):
            self._h = read_parity_check_matrix(source)
        else:
            self._h = sparse.csr_matrix(source, dtype=np.int32)
        self._n = self._h.shape[1]
        self._m = self._h.shape[0]
        self._k = self._n - self._m
        if self._n == 0:
            raise ValueError("Invalid parity check matrix: matrix is empty")
        self._rate = float(self._k) / self._n
        self._h_std, self._permutation = build_standard_form(self._h)
        rank = self._h_std.shape[0]
        if rank != self._m:  # encoder_decoder_data.py:280-305
            print(f"Warning: Matrix rank is {rank}, expected {self._m}. Some rows are linearly dependent.")
            self._m = rank
            self._k = self._n - self._m
            self._rate = float(self._k) / self._n
        self._h_sparse_cached = self._h_std
        # G^T = [I_k ; A] so that c = G^T u = [u, A u mod 2] (:319-344, data_buffer.py:47-82)
        A = self._h_std[:, : self._k]
        self._g_transpose = sparse.vstack([sparse.identity(self._k, dtype=np.int32, format="csr"),
                                           A]).tocsr().astype(np.int32)
        self._decoder_structures_initialized = False

    def physical_matrix(self):
        """H[:, perm]: the sparse ALIST graph in H_std's column order (same code;
        row operations do not change the null space) -- physical mode, §8 f4."""
        Hp = sparse.csr_matrix(self._h)[:, self._permutation].tocsr()
        Hp.sort_indices()
        return Hp

    # reference-compatible accessors
    def get_decoder_structures(self):
        coo = self._h_std.tocoo()
        return coo, None, None

    def encode(self, u):
        """[B, k] bits -> [B, n] codewords in H_std order (host helper for tests)."""
        u = np.atleast_2d(np.asarray(u, dtype=np.int64))
        par = (self._h_std[:, : self._k] @ u.T).T % 2
        return np.concatenate([u, par], axis=1).astype(np.uint8)


def load_committed_code(name, codes_dir=None):
    """Load a code shipped in ldpc_amd/codes (no ALIST file needed on the GPU box)."""
    codes_dir = codes_dir or CODES_DIR
    z = np.load(os.path.join(codes_dir, f"{name}.npz"), allow_pickle=False)
    m, n = int(z["m"]), int(z["n"])
    H = sparse.csr_matrix((z["h_data"], z["h_indices"], z["h_indptr"]), shape=(m, n))
    return EncoderDecoderData(H)
