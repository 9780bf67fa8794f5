// phys_kernels.hip -- "physical mode" SPA decoder, gfx950.
//
// NOT the reference's arithmetic (that is spa_kernels.hip, fp64 on H_std):
// this mode decodes the sparse ALIST graph H[:, perm] (same code, same column
// order as H_std -- row operations do not change the null space), with the LLR
// sign convention made consistent with the tanh rule (Lambda = log P0/P1 =
// -channel LLR, the reference's channel maps bit 1 to +LLR, channel.py:49,80),
// in fp32, every frame's whole state resident in LDS.  It has no reference
// parity by construction; tests compare it with its own CPU
// restatement (oracle/phys_oracle.c) and check that it decodes.
//
// Check update in the phi domain (phi(x) = -log tanh(x/2), self-inverse):
//   E[r,c] = sign * phi( sum_{c' in r} phi(|M[r,c']|) - phi(|M[r,c]|) ),
//   sign   = prod_{c' != c} sign(M[r,c']),   M[r,c] = L[c] - E[r,c]
// Variable update: L[c] = Lambda[c] + sum_r E[r,c].  Flooding schedule; early
// termination when H b = 0 with b = (L < 0); at most max_iter iterations.
//
// One workgroup (256 threads) per frame, frames grid-strided; LDS holds
// E[nnz], L[n], Lambda[n] in fp32 (<= 42 KB for the WiMAX 2304 codes: three
// frames per CU).  Threads own checks in the CN phase and columns in the VN
// phase; two barriers per iteration plus one OR-barrier for the syndrome.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "phys_math.h"
#include "spa_device.h"

namespace ldpc {
namespace {

struct PhysArgs {
    DevGraph g;               // H[:, perm] (sparse)
    const double *llr;        // [count][n] (layout 0) or ch tile layout (layout 1)
    int layout;               // 0: row per frame; 1: [tile][n][64] (on-device frames)
    int count;
    int max_iter;
    uint8_t *z_out;           // [count][n] or null: z = (bit estimate) ^ 1
    int *conv_out;            // [count] or null
    int *status_out;          // [count] or null
    int *iters_out;           // [count] or null
    float *post_out;          // [count][n] or null
    const uint32_t *ubits;    // MC: info bits [tile][kw][64] (layout 1), else null
    unsigned long long *ctr;  // MC: counters [7] or null
};

__global__ __launch_bounds__(256) void phys_kernel(PhysArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const DevGraph &g = a.g;
    float *E = lds;                 // [nnz]
    float *L = E + ((g.nnz + 3) & ~3);  // [n]
    float *Lam = L + ((g.n + 3) & ~3);  // [n]
    __shared__ int s_err;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int f = blockIdx.x; f < a.count; f += gridDim.x) {
        // --- load the frame: Lambda = -channel LLR
        for (int j = tid; j < g.n; j += nt) {
            const double ch = a.layout == 0 ? a.llr[(size_t)f * g.n + j]
                                            : a.llr[((size_t)(f >> 6) * g.n + j) * kTile + (f & 63)];
            Lam[j] = -(float)ch;
            L[j] = Lam[j];
        }
        for (int e = tid; e < g.nnz; e += nt) E[e] = 0.0f;
        __syncthreads();
        int conv = -1, it = 0;
        for (; it < a.max_iter; ++it) {
            // --- check nodes
            for (int r = tid; r < g.m; r += nt) {
                const int b = g.row_ptr[r], e1 = g.row_ptr[r + 1];
                float S = 0.0f;
                unsigned neg = 0u;
                for (int e = b; e < e1; ++e) {
                    const float M = L[g.col_idx[e]] - E[e];
                    S += phi(fabsf(M));
                    neg ^= (M < 0.0f) ? 1u : 0u;
                }
                for (int e = b; e < e1; ++e) {
                    const float M = L[g.col_idx[e]] - E[e];
                    const float mag = phi(fmaxf(S - phi(fabsf(M)), 0.0f));
                    E[e] = ((neg ^ ((M < 0.0f) ? 1u : 0u)) != 0u) ? -mag : mag;
                }
            }
            __syncthreads();
            // --- variable nodes
            for (int j = tid; j < g.n; j += nt) {
                float s = Lam[j];
                for (int p = g.csc_ptr[j]; p < g.csc_ptr[j + 1]; ++p) s += E[g.csc_edge[p]];
                L[j] = s;
            }
            __syncthreads();
            // --- syndrome of b = (L < 0)
            int bad = 0;
            for (int r = tid; r < g.m && !bad; r += nt) {
                unsigned par = 0u;
                for (int e = g.row_ptr[r]; e < g.row_ptr[r + 1]; ++e) par ^= (L[g.col_idx[e]] < 0.0f) ? 1u : 0u;
                bad = (int)par;
            }
            if (!__syncthreads_or(bad)) {
                conv = it;
                break;
            }
        }
        const int iters = conv >= 0 ? conv + 1 : a.max_iter;
        // --- outputs
        for (int j = tid; j < g.n; j += nt) {
            const bool bit = L[j] < 0.0f;
            if (a.z_out) a.z_out[(size_t)f * g.n + j] = bit ? 0 : 1;
            if (a.post_out) a.post_out[(size_t)f * g.n + j] = L[j];
        }
        if (tid == 0) {
            if (a.conv_out) a.conv_out[f] = conv;
            if (a.status_out) a.status_out[f] = conv >= 0 ? 0 : 1;
            if (a.iters_out) a.iters_out[f] = iters;
            s_err = 0;
        }
        if (a.ctr) {
            __syncthreads();
            if (conv < 0) {  // BER counts failed frames only (main.py:130-138)
                const int kw = (g.k + 31) >> 5;
                int my = 0;
                for (int j = tid; j < g.k; j += nt) {
                    const uint32_t w = a.ubits[((size_t)(f >> 6) * kw + (j >> 5)) * kTile + (f & 63)];
                    my += (((w >> (j & 31)) & 1u) != (L[j] < 0.0f ? 1u : 0u)) ? 1 : 0;
                }
                atomicAdd(&s_err, my);
            }
            __syncthreads();
            if (tid == 0) {
                atomicAdd(&a.ctr[0], 1ull);
                if (conv < 0) {
                    atomicAdd(&a.ctr[1], 1ull);
                    atomicAdd(&a.ctr[2], (unsigned long long)s_err);
                } else {
                    atomicAdd(&a.ctr[3], (unsigned long long)conv);
                    atomicAdd(&a.ctr[4], 1ull);
                }
                atomicAdd(&a.ctr[6], (unsigned long long)iters);
            }
        }
        __syncthreads();  // LDS reused by the next frame
    }
}

}  // namespace

size_t phys_lds_bytes(const DevGraph &g) {
    return sizeof(float) * (size_t)(((g.nnz + 3) & ~3) + 2 * ((g.n + 3) & ~3));
}

hipError_t launch_phys(const DevGraph &g, const double *llr, int layout, int count, int max_iter, uint8_t *z,
                       int *conv, int *status, int *iters, float *post, const uint32_t *ubits,
                       unsigned long long *ctr, int grid, hipStream_t s) {
    PhysArgs a{g, llr, layout, count, max_iter, z, conv, status, iters, post, ubits, ctr};
    const size_t lds = phys_lds_bytes(g);
    if (count > 0) phys_kernel<<<grid, 256, lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace ldpc
