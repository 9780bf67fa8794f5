"""ALIST parity-check matrix reader (input format of the decoder path).

Mirrors python_ldpc_app/utils.py:read_parity_check_matrix (lines 21-113):
line 1 ``N M`` (columns, rows); line 2 max weights (skipped); line 3 the N
column weights; line 4 the M row weights; then N column lines (skipped) and M
row lines of 1-based column indices where ``0`` is padding.  An empty row line
counts as a row with no entries (:84-87).  On any error the reference prints
the error and returns an EMPTY matrix (:109-113); ``read_parity_check_matrix``
does the same, and ``EncoderDecoderData`` turns that into ValueError.
"""
import sys

import numpy as np
from scipy import sparse


class AlistError(ValueError):
    pass


def _ints(line):
    return [int(x) for x in line.split() if x.strip()] if line and line.strip() else []


def parse_alist(text_lines):
    """Parse ALIST lines -> scipy CSR (int32).  Raises AlistError on bad input."""
    it = iter(text_lines)

    def nxt(what):
        try:
            return next(it)
        except StopIteration:
            raise AlistError(f"Unexpected end of file: {what}") from None

    first = nxt("missing dimensions").strip()
    if not first:
        raise AlistError("Empty file or missing dimensions")
    sizes = _ints(first)
    if len(sizes) < 2:
        raise AlistError("Invalid format: missing dimensions")
    n_cols, n_rows = sizes[0], sizes[1]
    if n_cols <= 0 or n_rows <= 0:
        raise AlistError(f"Invalid dimensions: cols={n_cols}, rows={n_rows}")
    nxt("missing max weights")
    col_w = _ints(nxt("missing column weights"))
    if len(col_w) != n_cols:
        raise AlistError(f"Column weights count mismatch: expected {n_cols}, got {len(col_w)}")
    row_w = _ints(nxt("missing row weights"))
    if len(row_w) != n_rows:
        raise AlistError(f"Row weights count mismatch: expected {n_rows}, got {len(row_w)}")
    for c in range(n_cols):
        nxt(f"while reading column {c}")
    rows, cols = [], []
    for r in range(len(row_w)):
        line = nxt(f"while reading row {r}").strip()
        if not line:
            continue
        for idx in _ints(line):
            if idx == 0:
                continue
            if idx < 1 or idx > n_cols:
                raise AlistError(f"Invalid column index {idx} in row {r} (valid range: 1-{n_cols})")
            rows.append(r)
            cols.append(idx - 1)
    data = np.ones(len(rows), dtype=np.int32)
    return sparse.coo_matrix((data, (rows, cols)), shape=(n_rows, n_cols), dtype=np.int32).tocsr()


def read_parity_check_matrix(file_name):
    """Reference-compatible reader: CSR on success, an empty 0x0 CSR on error."""
    try:
        with open(file_name, "r") as fh:
            return parse_alist(fh)
    except Exception as e:  # noqa: BLE001 - the reference swallows every error (:109-113)
        print(f"Error: Could not read parity check matrix from file {file_name}: {e}", file=sys.stderr)
        return sparse.csr_matrix((0, 0), dtype=np.int32)


def write_alist(H, file_name):
    """Write a CSR matrix as ALIST (used to round-trip the committed codes)."""
    H = sparse.csr_matrix(H)
    m, n = H.shape
    Hc = H.tocsc()
    cw = np.diff(Hc.indptr)
    rw = np.diff(H.indptr)
    with open(file_name, "w") as fh:
        fh.write(f"{n} {m}\n{int(cw.max(initial=0))} {int(rw.max(initial=0))}\n")
        fh.write(" ".join(map(str, cw)) + " \n")
        fh.write(" ".join(map(str, rw)) + " \n")
        for j in range(n):
            ids = sorted(Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]] + 1)
            fh.write(" ".join(map(str, ids)) + " \n")
        for i in range(m):
            ids = sorted(H.indices[H.indptr[i]:H.indptr[i + 1]] + 1)
            fh.write(" ".join(map(str, ids)) + " \n")
