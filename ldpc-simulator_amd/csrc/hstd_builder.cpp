// hstd_builder.cpp -- GF(2) standard form H_std = [A | I_m] on bit-packed rows.
//
// Replaces the reference's pure-Python Gauss-Jordan (about 44 s at n=2304,
// SURVEY.md §0.7) with a word-parallel one:
//   gaussian_elimination             encoder_decoder_data.py:13-183
//   create_standart_parity_check_matrix                    :269-317
// The pivot rule is the reference's: columns are scanned 0..n-1; the pivot is
// the first row >= cur_row holding a 1 (:46-49); rows are swapped (:57-63);
// rows BELOW are eliminated (:81-119); the scan stops once every row has a
// pivot (:124-125); back-elimination clears rows above each pivot (:130-176).
// Reduced row-echelon form is unique for a fixed pivot rule, so the result is
// the reference's H_std exactly (pinned by sha256 in tests/golden/codes).
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ldpc_internal.h"

struct ldpc_hstd {
    int32_t m_std = 0, n = 0;
    std::vector<int32_t> row_ptr, col_idx, perm;
};

namespace {

using word = uint64_t;

struct BitRows {
    int rows, cols, words;
    std::vector<word> bits;
    BitRows(int r, int c) : rows(r), cols(c), words((c + 63) / 64), bits((size_t)r * ((c + 63) / 64), 0) {}
    word *row(int r) { return bits.data() + (size_t)r * words; }
    bool get(int r, int c) const { return (bits[(size_t)r * words + (c >> 6)] >> (c & 63)) & 1u; }
    void xor_into(int dst, int src) {
        word *d = row(dst);
        const word *s = row(src);
        for (int w = 0; w < words; ++w) d[w] ^= s[w];
    }
    void swap_rows(int a, int b) {
        word *x = row(a), *y = row(b);
        for (int w = 0; w < words; ++w) std::swap(x[w], y[w]);
    }
};

// Forward elimination + back-substitution; returns the pivot ("successful") columns.
std::vector<int> gauss_jordan(BitRows &A) {
    const int nrows = A.rows, ncols = A.cols;
    std::vector<int> pivots;
    int cur_row = 0;
    for (int col = 0; col < ncols && cur_row < nrows; ++col) {
        int pr = -1;
        for (int r = cur_row; r < nrows; ++r)
            if (A.get(r, col)) { pr = r; break; }
        if (pr < 0) continue;  // dependent column (:51-54)
        if (pr > cur_row) A.swap_rows(pr, cur_row);
        for (int r = cur_row + 1; r < nrows; ++r)
            if (A.get(r, col)) A.xor_into(r, cur_row);
        pivots.push_back(col);
        if ((int)pivots.size() == nrows) break;
        ++cur_row;
    }
    for (int dc = 0; dc < (int)pivots.size(); ++dc) {
        const int col = pivots[dc];
        for (int r = 0; r < dc; ++r)
            if (A.get(r, col)) A.xor_into(r, dc);
    }
    return pivots;
}

}  // namespace

extern "C" int ldpc_hstd_build(int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                               ldpc_hstd **out) {
    if (!out) return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: out is NULL");
    *out = nullptr;
    if (m <= 0 || n <= 0 || !row_ptr || !col_idx)
        return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: empty matrix (m=%d n=%d)", m, n);
    if (row_ptr[0] != 0) return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: row_ptr[0] != 0");
    try {
        BitRows A(m, n);
        for (int r = 0; r < m; ++r) {
            if (row_ptr[r + 1] < row_ptr[r])
                return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: row_ptr not monotone at row %d", r);
            for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                const int c = col_idx[e];
                if (c < 0 || c >= n)
                    return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: column %d out of range in row %d", c, r);
                if (A.get(r, c))
                    return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_build: duplicate entry (%d,%d)", r, c);
                A.row(r)[c >> 6] |= word(1) << (c & 63);
            }
        }
        std::vector<int> piv = gauss_jordan(A);
        const int rank = (int)piv.size();
        // rank-deficient: keep the first `rank` rows (:280-305).  They are already
        // in reduced form, so re-running the elimination on them is the identity.
        auto *h = new ldpc_hstd;
        h->m_std = rank;
        h->n = n;
        std::vector<char> is_piv(n, 0);
        for (int c : piv) is_piv[c] = 1;
        h->perm.reserve(n);
        for (int c = 0; c < n; ++c)
            if (!is_piv[c]) h->perm.push_back(c);
        for (int c : piv) h->perm.push_back(c);
        // H_std[:, new] = RREF[:, perm[new]]  (matrix_sparse.py:128-163), CSR ascending
        h->row_ptr.assign(rank + 1, 0);
        for (int r = 0; r < rank; ++r) {
            for (int nc = 0; nc < n; ++nc)
                if (A.get(r, h->perm[nc])) h->col_idx.push_back(nc);
            h->row_ptr[r + 1] = (int32_t)h->col_idx.size();
        }
        *out = h;
        return LDPC_OK;
    } catch (const std::bad_alloc &) {
        return ldpc_fail(LDPC_ENOMEM, "ldpc_hstd_build: out of host memory");
    }
}

extern "C" int ldpc_hstd_get(const ldpc_hstd *h, int32_t *m_std, int32_t *n, int64_t *nnz,
                             const int32_t **row_ptr, const int32_t **col_idx, const int32_t **perm) {
    if (!h) return ldpc_fail(LDPC_EINVAL, "ldpc_hstd_get: NULL handle");
    if (m_std) *m_std = h->m_std;
    if (n) *n = h->n;
    if (nnz) *nnz = (int64_t)h->col_idx.size();
    if (row_ptr) *row_ptr = h->row_ptr.data();
    if (col_idx) *col_idx = h->col_idx.data();
    if (perm) *perm = h->perm.data();
    return LDPC_OK;
}

extern "C" void ldpc_hstd_free(ldpc_hstd *h) { delete h; }
