"""Native GF(2) standard-form builder (csrc/hstd_builder.cpp) vs the reference.

Pins: sha256 of H_std CSR and of the permutation, computed by the reference's
EncoderDecoderData (encoder_decoder_data.py:186-317) in ldpc_amd/codes.
"""
import numpy as np
import pytest
from scipy import sparse

import ldpc_amd
from conftest import load_code_npz

CODES = ["BCH_7_4_1_strip", "wimax_576_0.5", "wimax_2304_0.5", "wimax_2304_0.75A", "wimax_2304_0.75B"]


def _H(c):
    return sparse.csr_matrix((c["h_data"], c["h_indices"], c["h_indptr"]), shape=(int(c["m"]), int(c["n"])))


@pytest.mark.parametrize("name", CODES)
def test_hstd_matches_reference(name):
    c = load_code_npz(name)
    Hs, perm = ldpc_amd.build_standard_form(_H(c))
    assert Hs.shape == (int(c["m_std"]), int(c["n"]))
    assert Hs.nnz == int(c["hstd_nnz"])
    assert ldpc_amd.csr_fingerprint(Hs) == str(c["hstd_sha"])
    np.testing.assert_array_equal(np.asarray(perm), c["perm"])
    if "hstd_indices" in c.files:
        np.testing.assert_array_equal(Hs.indptr, c["hstd_indptr"])
        np.testing.assert_array_equal(Hs.indices, c["hstd_indices"])


@pytest.mark.parametrize("name", CODES)
def test_standard_form_structure(name):
    """H_std = [A | I_m] and H_std[:, j] = RREF(H)[:, perm[j]] spans the same code."""
    c = load_code_npz(name)
    H = _H(c)
    Hs, perm = ldpc_amd.build_standard_form(H)
    m, n = Hs.shape
    k = n - m
    ident = Hs[:, k:].toarray()
    np.testing.assert_array_equal(ident, np.eye(m, dtype=ident.dtype))
    # every codeword of H_std (in permuted order) is a codeword of H
    rng = np.random.default_rng(0)
    edd = ldpc_amd.EncoderDecoderData(H)
    u = rng.integers(0, 2, size=(8, k))
    cw_std = edd.encode(u)
    cw = np.zeros_like(cw_std)
    cw[:, perm] = cw_std
    assert not ((H @ cw.T.astype(np.int64)) % 2).any()
    assert not ((Hs @ cw_std.T.astype(np.int64)) % 2).any()


def test_rank_deficient_drops_rows():
    """encoder_decoder_data.py:280-305: keep the first `rank` rows, update m, k."""
    H = np.array([[1, 1, 0, 1, 0, 0],
                  [0, 1, 1, 0, 1, 0],
                  [1, 0, 1, 1, 1, 0],   # = row0 ^ row1
                  [0, 0, 0, 1, 1, 1]], dtype=np.int32)
    edd = ldpc_amd.EncoderDecoderData(sparse.csr_matrix(H))
    assert edd._m == 3 and edd._k == 3
    Hs = edd._h_std.toarray()
    np.testing.assert_array_equal(Hs[:, 3:], np.eye(3, dtype=Hs.dtype))


def test_pivot_rule_and_permutation_small():
    """Hand-checked: pivots are found left to right, first row >= cur_row."""
    H = np.array([[0, 1, 1, 0],
                  [1, 1, 0, 1]], dtype=np.int32)
    Hs, perm = ldpc_amd.build_standard_form(sparse.csr_matrix(H))
    # col 0 pivots on row 1 (swap), col 1 pivots on row 1 -> pivots [0, 1]
    # RREF = [[1,0,1,1],[0,1,1,0]]; perm = [2, 3, 0, 1]
    assert perm == [2, 3, 0, 1]
    np.testing.assert_array_equal(Hs.toarray(), np.array([[1, 1, 1, 0], [1, 0, 0, 1]]))


def test_rejects_duplicates_and_bad_columns():
    with pytest.raises(ldpc_amd.LdpcError):
        ldpc_amd.build_standard_form(sparse.csr_matrix(
            (np.ones(2, np.int32), np.array([1, 1]), np.array([0, 2])), shape=(1, 3)))


def test_empty_matrix_raises_like_reference(tmp_path):
    bad = tmp_path / "bad.alist"
    bad.write_text("")
    with pytest.raises(ValueError, match="empty"):
        ldpc_amd.EncoderDecoderData(str(bad))
