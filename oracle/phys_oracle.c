/*
 * phys_oracle.c -- CPU restatement of the physical-mode decoder
 * (ldpc-simulator_amd/csrc/phys_kernels.hip).  TEST INFRASTRUCTURE ONLY.
 *
 * This mode is OUR design, not the reference's arithmetic:
 * standard sum-product on the sparse graph H[:, perm], Lambda = -llr, fp32,
 * phi-domain check update, flooding, syndrome early termination.  Parity is
 * against this restatement (same operation order; expm1f/log1pf differ from
 * the GPU's at the ulp level, so tests compare decisions, not bits).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* the GPU evaluates the same formula on the hardware exp2 / rcp / log2 (phys_math.h):
   equal to this one to a few ulp, so tests compare decisions */
static float phi(float x) {
    x = fminf(fmaxf(x, 1.0e-7f), 30.0f);
    if (x < 0.03125f) return logf(2.0f * (1.0f / x)) + x * x * (1.0f / 12.0f);
    const float t = expf(x);
    return logf((t + 1.0f) * (1.0f / (t - 1.0f)));
}

int oracle_phys_decode(int m, int n, const int *row_ptr, const int *col_idx, int batch, const double *llr,
                       int max_iter, uint8_t *z_out, int *conv_out, int *iters_out, float *post_out) {
    if (m <= 0 || n <= 0 || max_iter < 1) return -1;
    const int nnz = row_ptr[m];
    int *cptr = (int *)calloc((size_t)n + 1, sizeof(int)), *cedge = (int *)malloc(sizeof(int) * (size_t)nnz);
    int *fill = (int *)malloc(sizeof(int) * (size_t)n);
    float *E = (float *)malloc(sizeof(float) * (size_t)nnz), *L = (float *)malloc(sizeof(float) * (size_t)n),
          *Lam = (float *)malloc(sizeof(float) * (size_t)n);
    if (!cptr || !cedge || !fill || !E || !L || !Lam) return -1;
    for (int e = 0; e < nnz; ++e) cptr[col_idx[e] + 1]++;
    for (int j = 0; j < n; ++j) cptr[j + 1] += cptr[j];
    memcpy(fill, cptr, sizeof(int) * (size_t)n);
    for (int r = 0; r < m; ++r)
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) cedge[fill[col_idx[e]]++] = e;
    for (int f = 0; f < batch; ++f) {
        for (int j = 0; j < n; ++j) L[j] = Lam[j] = -(float)llr[(size_t)f * n + j];
        memset(E, 0, sizeof(float) * (size_t)nnz);
        int conv = -1, it = 0;
        for (; it < max_iter; ++it) {
            for (int r = 0; r < m; ++r) {
                float S = 0.0f;
                unsigned neg = 0u;
                for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                    const float M = L[col_idx[e]] - E[e];
                    S += phi(fabsf(M));
                    neg ^= M < 0.0f ? 1u : 0u;
                }
                for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                    const float M = L[col_idx[e]] - E[e];
                    const float mag = phi(fmaxf(S - phi(fabsf(M)), 0.0f));
                    E[e] = (neg ^ (M < 0.0f ? 1u : 0u)) ? -mag : mag;
                }
            }
            for (int j = 0; j < n; ++j) {
                float s = Lam[j];
                for (int p = cptr[j]; p < cptr[j + 1]; ++p) s += E[cedge[p]];
                L[j] = s;
            }
            int bad = 0;
            for (int r = 0; r < m && !bad; ++r) {
                unsigned par = 0u;
                for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) par ^= L[col_idx[e]] < 0.0f ? 1u : 0u;
                bad = (int)par;
            }
            if (!bad) {
                conv = it;
                break;
            }
        }
        for (int j = 0; j < n; ++j) {
            if (z_out) z_out[(size_t)f * n + j] = L[j] < 0.0f ? 0 : 1;
            if (post_out) post_out[(size_t)f * n + j] = L[j];
        }
        if (conv_out) conv_out[f] = conv;
        if (iters_out) iters_out[f] = conv >= 0 ? conv + 1 : max_iter;
    }
    free(cptr);
    free(cedge);
    free(fill);
    free(E);
    free(L);
    free(Lam);
    return 0;
}
