"""SPA_Decoder's constructor validates H without touching HIP:
ldpc_amd.device.validate_csr restates ldpc_graph_create's argument checks
(csrc/ldpc_api.cpp:328-353), so a malformed matrix fails in the parent process
at construction, as the reference's constructor would (spa_decoder.py:16-42),
not on the first decode() inside a forked worker.  The C library runs the same
checks before it looks for a GPU, so on this CPU-only host both must reject
the same inputs with the same codes."""
import ctypes

import numpy as np
import pytest
from scipy import sparse

from ldpc_amd import _lib
from ldpc_amd.device import validate_csr
from ldpc_amd.spa_decoder import SPA_Decoder


class _Edd:
    def __init__(self, H):
        self._h_sparse_cached = sparse.csr_matrix(H)
        self._m, self._n = self._h_sparse_cached.shape


def _c_rc(m, n, indptr, indices):
    h = ctypes.c_void_p()
    ip = np.ascontiguousarray(indptr, np.int32)
    ix = np.ascontiguousarray(indices if len(indices) else [0], np.int32)
    return _lib.lib().ldpc_graph_create(m, n, _lib.i32p(ip), _lib.i32p(ix), -1, ctypes.byref(h))


CASES = {
    "ok": (2, 4, [0, 2, 4], [0, 2, 1, 3]),
    "m_gt_n": (3, 2, [0, 1, 2, 3], [0, 1, 0]),
    "row_ptr0": (2, 4, [1, 2, 4], [0, 2, 1, 3]),
    "not_monotone": (2, 4, [0, 3, 2], [0, 2, 3]),
    "col_range": (2, 4, [0, 2, 4], [0, 4, 1, 3]),
    "duplicate": (2, 4, [0, 2, 4], [1, 1, 0, 3]),
    "descending": (2, 4, [0, 2, 4], [0, 2, 3, 1]),
    "empty": (2, 4, [0, 0, 0], []),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_python_checks_equal_the_c_checks(name):
    m, n, ip, ix = CASES[name]
    rc = _c_rc(m, n, ip, ix)
    if name == "ok":
        validate_csr(m, n, np.array(ip), np.array(ix))
        assert rc in (0, -5)  # accepted: EDEVICE without a GPU
        return
    with pytest.raises(_lib.LdpcError) as ei:
        validate_csr(m, n, np.array(ip), np.array(ix))
    assert ei.value.code == rc, (name, rc)


class _Settings:
    def get_max_iterations(self):
        return 10

    def is_normalized_llr_calculate(self):
        return False


def test_constructor_fails_fast_without_hip():
    H = sparse.csr_matrix((np.ones(4), np.array([1, 1, 0, 3]), np.array([0, 2, 4])), shape=(2, 4))
    with pytest.raises(_lib.LdpcError, match="strictly ascending"):
        SPA_Decoder(_Edd(H), _Settings())
    with pytest.raises(ValueError):
        SPA_Decoder(_Edd(sparse.csr_matrix(np.array([[1, 0, 1, 0], [0, 1, 0, 1]]))), _Settings(), max_frames=0)
    dec = SPA_Decoder(_Edd(sparse.csr_matrix(np.array([[1, 0, 1, 0], [0, 1, 0, 1]]))), _Settings())
    assert dec._dev is None  # no HIP work at construction
