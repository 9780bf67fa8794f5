"""ALIST reader (ldpc_amd.alist) -- mirrors python_ldpc_app/utils.py:21-113."""
import os

import numpy as np
import pytest
from scipy import sparse

from ldpc_amd import alist
from conftest import load_code_npz

REF_DB = "/root/reference/Channel_Codes_Database"
NAMES = {
    "BCH_7_4_1_strip": "BCH_7_4_1_strip.alist.txt",
    "wimax_576_0.5": "Wimax LDPC Codes/wimax_576_0.5.alist.txt",
    "wimax_2304_0.5": "Wimax LDPC Codes/wimax_2304_0.5.alist.txt",
}


def _H(c):
    return sparse.csr_matrix((c["h_data"], c["h_indices"], c["h_indptr"]), shape=(int(c["m"]), int(c["n"])))


@pytest.mark.parametrize("name", sorted(NAMES))
def test_roundtrip_committed_codes(name, tmp_path):
    H = _H(load_code_npz(name))
    p = tmp_path / "c.alist"
    alist.write_alist(H, str(p))
    H2 = alist.read_parity_check_matrix(str(p))
    assert H2.shape == H.shape
    assert (H2 != H).nnz == 0


@pytest.mark.parametrize("name", sorted(NAMES))
def test_reads_reference_files_like_reference(name):
    """When the reference tree is present (build container), parse its ALIST
    files and compare with the CSR the reference reader produced (golden)."""
    path = os.path.join(REF_DB, NAMES[name])
    if not os.path.exists(path):
        pytest.skip("reference database not present (GPU box)")
    H = alist.read_parity_check_matrix(path)
    ref = _H(load_code_npz(name))
    np.testing.assert_array_equal(H.indptr, ref.indptr)
    np.testing.assert_array_equal(H.indices, ref.indices)


def test_bch_text():
    txt = ["7 3", "3 4", "1 1 2 2 3 2 1", "4 4 4", "1 0 0", "2 0 0", "1 3 0", "1 2 0", "1 2 3",
           "2 3 0", "3 0 0", "1 3 4 5", "2 4 5 6", "3 5 6 7"]
    H = alist.parse_alist(txt)
    np.testing.assert_array_equal(H.toarray(), [[1, 0, 1, 1, 1, 0, 0], [0, 1, 0, 1, 1, 1, 0], [0, 0, 1, 0, 1, 1, 1]])


@pytest.mark.parametrize("bad", [
    [],                                  # empty file
    ["7"],                               # missing dimension
    ["0 3"],                             # invalid dimension
    ["2 1", "1 2", "1 1 1", "2"],        # column weights count mismatch
    ["2 1", "1 2", "1 1", "2", "1", "1", "1 3"],  # column index out of range
    ["2 1", "1 2", "1 1", "2", "1"],     # truncated
])
def test_errors_return_empty_like_reference(bad, tmp_path):
    p = tmp_path / "x.alist"
    p.write_text("\n".join(bad) + ("\n" if bad else ""))
    H = alist.read_parity_check_matrix(str(p))
    assert H.shape == (0, 0)


def test_missing_file_returns_empty():
    assert alist.read_parity_check_matrix("/nonexistent/file.alist").shape == (0, 0)


def test_padding_zeros_and_blank_rows():
    txt = ["3 2", "2 2", "1 1 1", "2 1", "1", "1", "2", "1 2 0", ""]
    H = alist.parse_alist(txt)
    np.testing.assert_array_equal(H.toarray(), [[1, 1, 0], [0, 0, 0]])
