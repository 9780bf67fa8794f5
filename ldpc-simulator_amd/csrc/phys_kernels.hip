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
#include <cstdlib>

#include "phys_math.h"
#include "spa_device.h"

namespace ldpc {
namespace {

struct PhysArgs {
    DevGraph g;               // H[:, perm] (sparse)
    const double *llr;        // [count][n] (layout 0) or ch tile layout (layout 1)
    const float *lam;         // layout 2: [count][n] fp32 Lambda (on-device frames, frame_kernels.hip)
    int layout;               // 0: row per frame; 1: [tile][n][64]; 2: lam
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

// Frame f into LDS: Lambda = -channel LLR, L = Lambda, E = 0.
__device__ __forceinline__ void frame_load(const PhysArgs &a, int f, float *E, float *L, float *Lam, int tid,
                                           int nt) {
    const DevGraph &g = a.g;
    for (int j = tid; j < g.n; j += nt) {
        if (a.layout == 2) {
            Lam[j] = a.lam[(size_t)f * g.n + j];  // contiguous per frame
        } else {
            const double ch = a.layout == 0 ? a.llr[(size_t)f * g.n + j]
                                            : a.llr[((size_t)(f >> 6) * g.n + j) * kTile + (f & 63)];
            Lam[j] = -(float)ch;
        }
        L[j] = Lam[j];
    }
    for (int e = tid; e < g.nnz; e += nt) E[e] = 0.0f;
}

// Monte-Carlo counters of the frames one workgroup decodes (thread 0's
// registers), added to the device counters once, when the workgroup is done:
// one atomic per counter per frame on the same 7 addresses serialised every
// frame of a launch in L2.
struct FrameCounts {
    unsigned long long v[7] = {0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void flush(unsigned long long *ctr) const {
        if (!ctr) return;
#pragma unroll
        for (int i = 0; i < 7; ++i)
            if (v[i]) atomicAdd(&ctr[i], v[i]);
    }
};

// Outputs and Monte-Carlo counters of frame f (conv = -1: not converged).
__device__ __forceinline__ void frame_finish(const PhysArgs &a, int f, int conv, const float *L, int *s_err,
                                             int tid, int nt, FrameCounts &fc) {
    const DevGraph &g = a.g;
    const int iters = conv >= 0 ? conv + 1 : a.max_iter;
    for (int j = tid; j < g.n; j += nt) {
        const bool bit = L[j] < 0.0f;
        if (a.z_out) a.z_out[(size_t)f * g.n + j] = bit ? 0 : 1;
        if (a.post_out) a.post_out[(size_t)f * g.n + j] = L[j];
    }
    if (tid == 0) {
        if (a.conv_out) a.conv_out[f] = conv;
        if (a.status_out) a.status_out[f] = conv >= 0 ? 0 : 1;
        if (a.iters_out) a.iters_out[f] = iters;
        *s_err = 0;
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
            atomicAdd(s_err, my);
        }
        __syncthreads();
        if (tid == 0) {
            fc.v[0] += 1ull;
            if (conv < 0) {
                fc.v[1] += 1ull;
                fc.v[2] += (unsigned long long)*s_err;
            } else {
                fc.v[3] += (unsigned long long)conv;
                fc.v[4] += 1ull;
            }
            fc.v[6] += (unsigned long long)iters;
        }
    }
    __syncthreads();  // LDS reused by the next frame
}

__global__ __launch_bounds__(256) void phys_kernel(PhysArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const DevGraph &g = a.g;
    float *E = lds;                 // [nnz]
    float *L = E + ((g.nnz + 3) & ~3);  // [n]
    float *Lam = L + ((g.n + 3) & ~3);  // [n]
    __shared__ int s_err;
    FrameCounts fc;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int f = blockIdx.x; f < a.count; f += gridDim.x) {
        frame_load(a, f, E, L, Lam, tid, nt);
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
        frame_finish(a, f, conv, L, &s_err, tid, nt, fc);
    }
    if (tid == 0) fc.flush(a.ctr);
}

// The same decoder with every thread's rows and columns fixed for the whole
// launch (row r = tid + k*NT, column j = tid + k*NT), their column indices and
// CSC edge ids held in registers as 16-bit pairs (loaded once, reused for every
// frame: no index loads in the iteration loop), and phi(|M|) kept in registers
// between the two sweeps of a row (phys_cn_tile does the same).  Identical
// operations in identical order as phys_kernel: bit-identical results.
template <int NT, int RPT, int RDEG, int CPT, int CDEG, int WPS>
__global__ __launch_bounds__(NT, WPS) void phys_reg_kernel(PhysArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const DevGraph &g = a.g;
    float *E = lds;
    float *L = E + ((g.nnz + 3) & ~3);
    float *Lam = L + ((g.n + 3) & ~3);
    __shared__ int s_err;
    FrameCounts fc;
    const int tid = threadIdx.x;
    int rbeg[RPT], rdeg[RPT];
    uint32_t rc[RPT][RDEG / 2];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = tid + k * NT;
        rbeg[k] = r < g.m ? g.row_ptr[r] : 0;
        rdeg[k] = r < g.m ? g.row_ptr[r + 1] - rbeg[k] : 0;
#pragma unroll
        for (int i = 0; i < RDEG / 2; ++i) {
            const uint32_t lo = 2 * i < rdeg[k] ? (uint32_t)g.col_idx[rbeg[k] + 2 * i] : 0u;
            const uint32_t hi = 2 * i + 1 < rdeg[k] ? (uint32_t)g.col_idx[rbeg[k] + 2 * i + 1] : 0u;
            rc[k][i] = lo | (hi << 16);
        }
    }
    int cdeg[CPT];
    uint32_t ce[CPT][CDEG / 2];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const int j = tid + k * NT;
        const int p0 = j < g.n ? g.csc_ptr[j] : 0;
        cdeg[k] = j < g.n ? g.csc_ptr[j + 1] - p0 : 0;
#pragma unroll
        for (int i = 0; i < CDEG / 2; ++i) {
            const uint32_t lo = 2 * i < cdeg[k] ? (uint32_t)g.csc_edge[p0 + 2 * i] : 0u;
            const uint32_t hi = 2 * i + 1 < cdeg[k] ? (uint32_t)g.csc_edge[p0 + 2 * i + 1] : 0u;
            ce[k][i] = lo | (hi << 16);
        }
    }
    auto col = [&](int k, int i) -> int { return (int)((rc[k][i >> 1] >> ((i & 1) * 16)) & 0xffffu); };
    auto edge = [&](int k, int i) -> int { return (int)((ce[k][i >> 1] >> ((i & 1) * 16)) & 0xffffu); };

    for (int f = blockIdx.x; f < a.count; f += gridDim.x) {
        frame_load(a, f, E, L, Lam, tid, NT);
        __syncthreads();
        int conv = -1;
        for (int it = 0; it < a.max_iter; ++it) {
            // --- check nodes
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                if (rdeg[k] == 0) continue;
                float ph[RDEG];
                uint32_t sg = 0u;
                float S = 0.0f;
#pragma unroll
                for (int i = 0; i < RDEG; ++i) {
                    if (i < rdeg[k]) {
                        const float M = L[col(k, i)] - E[rbeg[k] + i];
                        ph[i] = phi(fabsf(M));
                        S += ph[i];
                        sg |= (M < 0.0f ? 1u : 0u) << i;
                    }
                }
                const uint32_t neg = __popc(sg) & 1u;
#pragma unroll
                for (int i = 0; i < RDEG; ++i) {
                    if (i < rdeg[k]) {
                        const float mag = phi(fmaxf(S - ph[i], 0.0f));
                        E[rbeg[k] + i] = ((neg ^ (sg >> i)) & 1u) ? -mag : mag;
                    }
                }
            }
            __syncthreads();
            // --- variable nodes
#pragma unroll
            for (int k = 0; k < CPT; ++k) {
                const int j = tid + k * NT;
                if (j >= g.n) continue;
                float s = Lam[j];
#pragma unroll
                for (int i = 0; i < CDEG; ++i)
                    if (i < cdeg[k]) s += E[edge(k, i)];
                L[j] = s;
            }
            __syncthreads();
            // --- syndrome of b = (L < 0)
            uint32_t bad = 0u;
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                uint32_t par = 0u;
#pragma unroll
                for (int i = 0; i < RDEG; ++i)
                    if (i < rdeg[k]) par ^= (L[col(k, i)] < 0.0f) ? 1u : 0u;
                bad |= par;
            }
            if (!__syncthreads_or((int)bad)) {
                conv = it;
                break;
            }
        }
        frame_finish(a, f, conv, L, &s_err, tid, NT, fc);
    }
    if (tid == 0) fc.flush(a.ctr);
}

}  // namespace

size_t phys_lds_bytes(const DevGraph &g) {
    return sizeof(float) * (size_t)(((g.nnz + 3) & ~3) + 2 * ((g.n + 3) & ~3));
}

namespace {

// Shape of phys_reg_kernel for this graph (0 = none: the generic phys_kernel).
// LDPC_PHYS_REG=0 forces phys_kernel (A/B).
struct RegShape {
    int rpt, rdeg, cpt, cdeg;
};
constexpr int kRegNT = 512;
constexpr RegShape kRegShapes[] = {{1, 8, 1, 8}, {1, 8, 2, 8}, {2, 8, 3, 8}, {2, 16, 5, 8}, {3, 8, 5, 8}};

int reg_shape(const DevGraph &g) {
    static const int force = [] {
        const char *e = getenv("LDPC_PHYS_REG");
        return e ? atoi(e) : -1;
    }();
    if (force == 0 || g.nnz >= 65536 || g.n >= 65536) return -1;  // 16-bit indices
    const int mc = g.max_col_deg;
    const int rpt = (g.m + kRegNT - 1) / kRegNT, cpt = (g.n + kRegNT - 1) / kRegNT;
    int best = -1;
    for (int i = 0; i < (int)(sizeof(kRegShapes) / sizeof(kRegShapes[0])); ++i) {
        const RegShape &r = kRegShapes[i];
        if (r.rpt >= rpt && r.cpt >= cpt && r.rdeg >= g.max_row_deg && r.cdeg >= mc &&
            (best < 0 || r.rpt * r.rdeg + r.cpt * r.cdeg <
                             kRegShapes[best].rpt * kRegShapes[best].rdeg + kRegShapes[best].cpt * kRegShapes[best].cdeg))
            best = i;
    }
    return best;
}

}  // namespace

int phys_block_threads(const DevGraph &g) { return reg_shape(g) >= 0 ? kRegNT : 256; }

hipError_t launch_phys(const DevGraph &g, const double *llr, const float *lam, int layout, int count, int max_iter,
                       uint8_t *z, int *conv, int *status, int *iters, float *post, const uint32_t *ubits,
                       unsigned long long *ctr, int grid, hipStream_t s) {
    PhysArgs a{g, llr, lam, layout, count, max_iter, z, conv, status, iters, post, ubits, ctr};
    const size_t lds = phys_lds_bytes(g);
    if (count <= 0) return hipSuccess;
    // min waves per SIMD of the large shapes: 6 = three 8-wave frames per CU (the
    // LDS limit for the 2304 codes) with a few spills beat 4 = two frames without
    // (tools/ab_physreg.sh: 2304 r1/2 -2.5 dB 51.9 vs 59.2 ms); LDPC_PHYS_REG_WPS=4 (A/B)
    static const int wps = [] {
        const char *e = getenv("LDPC_PHYS_REG_WPS");
        return e ? atoi(e) : 6;
    }();
    switch (reg_shape(g)) {
    case 0: phys_reg_kernel<kRegNT, 1, 8, 1, 8, 6><<<grid, kRegNT, lds, s>>>(a); break;
    case 1: phys_reg_kernel<kRegNT, 1, 8, 2, 8, 6><<<grid, kRegNT, lds, s>>>(a); break;
    case 2:
        if (wps == 6) phys_reg_kernel<kRegNT, 2, 8, 3, 8, 6><<<grid, kRegNT, lds, s>>>(a);
        else phys_reg_kernel<kRegNT, 2, 8, 3, 8, 4><<<grid, kRegNT, lds, s>>>(a);
        break;
    case 3:
        if (wps == 6) phys_reg_kernel<kRegNT, 2, 16, 5, 8, 6><<<grid, kRegNT, lds, s>>>(a);
        else phys_reg_kernel<kRegNT, 2, 16, 5, 8, 4><<<grid, kRegNT, lds, s>>>(a);
        break;
    case 4:
        if (wps == 6) phys_reg_kernel<kRegNT, 3, 8, 5, 8, 6><<<grid, kRegNT, lds, s>>>(a);
        else phys_reg_kernel<kRegNT, 3, 8, 5, 8, 4><<<grid, kRegNT, lds, s>>>(a);
        break;
    default: phys_kernel<<<grid, 256, lds, s>>>(a);
    }
    return hipGetLastError();
}

}  // namespace ldpc
