// edge_kernels.hip -- the few-frame decode path (gfx950): lanes over a row's or
// a column's EDGES instead of over frames.
//
// main.py calls decode() once per frame (python_ldpc_app/main.py:124,312), and
// the drop-in SPA_Decoder keeps that: one frame per call.  Every other kernel
// of this library puts one frame per lane, so a call on one frame runs each
// check row as a single wavefront walking the row's ~600 edges with a few
// loads in flight -- 1.6 ms per CN pass and 2 ms per iteration whatever the
// frame count (profiles/r3g_small).  Here a wavefront takes one (tile, row)
// (or (tile, column)) and its lanes take contiguous pieces of the row's edges
// (lane l: positions [l*KE, l*KE + KE)), frame after frame over the tile's
// live frames, so all of a row's loads are in flight at once and tanh / the
// quotients run across lanes.  The arithmetic and its order are the
// reference's and the other kernels' (spa_decoder.py:112-185):
//   cn_edge_kernel  M = L[col] - E_old (iteration 0: M = ch), t = tanh(M/2)
//                   clipped (:138-146); P = t0*t1*... strictly left to right:
//                   lane 0 multiplies its pieces into the running product,
//                   which moves to lane 1 (two readlanes), ... (:151-152);
//                   q = P/t, or for |t| <= 1e-10 the in-order product of the
//                   others (:159-164, cn_rare_kernel's case, done here);
//                   E_new = 2 atanh(clip(q)) (:167-168)
//   vn_edge_kernel  S = ((0 + E_r0) + E_r1) + ... rows ascending, passed lane
//                   to lane the same way; L = ch + S (:173-185), z^1 bit,
//                   normalized-LLR count (:210-228): vn_cols_kernel's outputs
//   syn_kernel      row parities popcount(A_r & (z^1)_A) + (z^1)_{k+r}
//                   (:191-204) over many workgroups (lane = frame), OR-ed
//                   into a per-frame flag that tail_exit_kernel then reads;
//                   syn_row_kernel (<= 4 frames): the same with lane = row
// Bit-identical to the split path (tests/test_gpu_edge.py).  Used by
// ldpc_decode_f64 for batches of at most LDPC_EDGE_FRAMES frames (ldpc_api.cpp).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cn_common.h"
#include "spa_device.h"
#include "spa_math.h"

namespace ldpc {
namespace {

constexpr int kEdgeKE = 16;  // edges per lane: rows and columns of up to 1,024 edges
constexpr int kSynRows = 8;  // rows per wavefront of syn_kernel
constexpr int kSynKw = 64;   // (z^1)_A words per lane: k <= 2048 (the column-parallel path's limit)

__device__ __forceinline__ double readlane_d(double x, int l) {
    const uint64_t u = dbits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return dfrom(((uint64_t)hi << 32) | lo);
}

// KE: edges per lane, fixed per graph (ceil(max_row_deg / 64) rounded up to
// 4, 8, 12 or 16) so every slot loop is static: a row-dependent count made the
// compiler keep a guard per slot and spill SGPRs to VGPR lanes.
template <bool kFirst, int KE>
__global__ __launch_bounds__(256) void cn_edge_kernel(DevGraph g, DevState st, AtanhCoef ac) {
    __shared__ MathLds mlds;
    const int tile = blockIdx.y;
    if (!st.tile_active[tile]) return;  // block-uniform
    fill_math_lds(mlds);
    __syncthreads();
    const LdsTanh ttab{mlds.tanh};
    const LdsAtanh ltab{mlds.atanh};
    const int lane = threadIdx.x & 63;
    const int row = (int)blockIdx.x * 4 + uniform(threadIdx.x >> 6);
    if (row >= g.m) return;
    const int beg = g.row_ptr[row], deg = g.row_ptr[row + 1] - beg;
    if (deg == 0) return;  // spa_decoder.py:115-122
    const int nlanes = (deg + KE - 1) / KE;  // lanes holding edges (deg <= 64 KE: host check)
    const int p0 = lane * KE;
    const int nl = max(0, min(deg - p0, KE));  // this lane's edges; slots past them repeat the last edge
    int col[KE];
#pragma unroll
    for (int i = 0; i < KE; ++i) col[i] = g.col_idx[beg + min(p0 + i, deg - 1)];
    unsigned long long live = __ballot(st.done[tile * kTile + lane] == 0);
    while (live != 0ull) {
        const int f = __ffsll((long long)live) - 1;  // uniform
        live &= live - 1ull;
        double *Ef = st.E + e_base(g, tile, f);
        const double *Lf = (kFirst ? st.ch : st.L) + (size_t)tile * g.n * kTile + f;
        double t[KE];
#pragma unroll
        for (int i = 0; i < KE; ++i) {
            double M = Lf[(size_t)col[i] * kTile];
            if (!kFirst) M = M - Ef[(size_t)(beg + min(p0 + i, deg - 1)) * g.ef];  // :260-268
            t[i] = M;
        }
        uint32_t tiny = 0u;  // this lane's slots with |t| <= 1e-10
#pragma unroll
        for (int i = 0; i < KE; ++i) {
            t[i] = cn_tanh(t[i], ttab);
            if (i < nl && !(fabs(t[i]) > kTiny)) tiny |= 1u << i;
        }
        // P = t0 * t1 * ... left to right (1.0 * t0 == t0 exactly)
        double P = 1.0;
        for (int l = 0; l < nlanes; ++l) {
            double x = P;
            if (lane == l) {
#pragma unroll
                for (int i = 0; i < KE; ++i)
                    if (i < nl) x = x * t[i];
            }
            P = readlane_d(x, l);
        }
        double En[KE];
        if (__ballot(tiny != 0u) == 0ull) {
            // q = P/t (div_nr: the IEEE quotient when P is not tiny, cn_common.h);
            // E_new = 2 atanh(clip(q)), or 2q where every quotient of the
            // wavefront is below 2^-27 (exact: spa_math.h kAtanhIdent)
            const bool nr = div_nr_ok(P);
#pragma unroll
            for (int i = 0; i < KE; ++i) {
                const double q = nr ? div_nr(P, t[i]) : P / t[i];
                En[i] = __ballot(!(fabs(q) < kAtanhIdent)) == 0ull ? 2.0 * q : 2.0 * atanh_f(clip_cl(q), ltab, ac);
            }
        } else {
            // rare (cn_rare_kernel's arithmetic): q = P/t, and for an edge with
            // |t| <= 1e-10 the in-order product of the others (:164)
#pragma unroll
            for (int i = 0; i < KE; ++i) En[i] = 2.0 * atanh_f(clip_cl(P / t[i]), ltab, ac);
            unsigned long long tl = __ballot(tiny != 0u);
            while (tl != 0ull) {
                const int lp = __ffsll((long long)tl) - 1;  // uniform
                tl &= tl - 1ull;
                uint32_t tm = (uint32_t)__builtin_amdgcn_readlane((int)tiny, lp);
                while (tm != 0u) {
                    const int ip = __ffs((int)tm) - 1;  // uniform
                    tm &= tm - 1u;
                    double q = 1.0;  // np.prod of the others (1.0 * t == t exactly; empty: 1.0)
                    for (int l = 0; l < nlanes; ++l) {
                        double x = q;
                        if (lane == l) {
#pragma unroll
                            for (int i = 0; i < KE; ++i)
                                if (i < nl && !(l == lp && i == ip)) x = x * t[i];
                        }
                        q = readlane_d(x, l);
                    }
                    if (lane == lp) {
                        const double v = 2.0 * atanh_f(clip_cl(q), ltab, ac);
#pragma unroll
                        for (int i = 0; i < KE; ++i)
                            if (i == ip) En[i] = v;
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < KE; ++i)
            if (i < nl) Ef[(size_t)(beg + p0 + i) * g.ef] = En[i];
    }
}

// One wavefront per (tile, column j), lanes over the column's edges (CSC
// order: rows ascending), frame after frame: vn_cols_kernel's results.
template <int KV>
__global__ __launch_bounds__(256) void vn_edge_kernel(DevGraph g, DevState st, int nllr, uint32_t *zb, int *cnt,
                                                      int first) {
    const int tile = blockIdx.y;
    const int j = (int)blockIdx.x * 4 + uniform(threadIdx.x >> 6);
    if (j >= g.n || !st.tile_active[tile]) return;
    const int lane = threadIdx.x & 63;
    const int p0 = g.csc_ptr[j], dc = g.csc_ptr[j + 1] - p0;
    const int nlanes = (dc + KV - 1) / KV;  // (dc <= 64 KV: host check)
    const int q0 = lane * KV;
    const int nl = max(0, min(dc - q0, KV));
    int ed[KV];
#pragma unroll
    for (int i = 0; i < KV; ++i) ed[i] = dc > 0 ? g.csc_edge[p0 + min(q0 + i, dc - 1)] : 0;
    const int nw = (g.n + 31) >> 5;
    unsigned long long live = __ballot(st.done[tile * kTile + lane] == 0);
    while (live != 0ull) {
        const int f = __ffsll((long long)live) - 1;  // uniform
        live &= live - 1ull;
        const double *Ef = st.E + e_base(g, tile, f);
        double v[KV];
#pragma unroll
        for (int i = 0; i < KV; ++i) v[i] = dc > 0 ? Ef[(size_t)ed[i] * g.ef] : 0.0;
        double s = 0.0;  // rows ascending, starting at 0.0
        for (int l = 0; l < nlanes; ++l) {
            double x = s;
            if (lane == l) {
#pragma unroll
                for (int i = 0; i < KV; ++i)
                    if (i < nl) x = x + v[i];
            }
            s = readlane_d(x, l);
        }
        if (lane == 0) {
            const size_t ci = ((size_t)tile * g.n + j) * kTile + f;
            const double chj = st.ch[ci];
            const double Lj = chj + s;  // channel added after the sum
            if (nllr && j < g.k) {
                const double ap = first ? chj : st.L[ci];  // previous posterior (ch on iteration 0)
                if (fabs(Lj) <= 7.0 && ap * Lj < 0.0) atomicAdd(&cnt[tile * kTile + f], 1);
            }
            st.L[ci] = Lj;
            if (!(Lj < 0.0)) atomicOr(&zb[((size_t)tile * nw + (j >> 5)) * kTile + f], 1u << (j & 31));
        }
    }
}

// Row parities of the tile's frames (lane = frame) over kSynRows rows per
// wavefront; a frame with an odd row gets bad[f] |= 1 (tail_exit_kernel reads
// and clears it).
__global__ __launch_bounds__(256) void syn_kernel(DevGraph g, DevState st, const uint32_t *zb, int *bad) {
    const int tile = blockIdx.y;
    if (!st.tile_active[tile]) return;
    const int lane = threadIdx.x & 63;
    const int r0 = ((int)blockIdx.x * 4 + uniform(threadIdx.x >> 6)) * kSynRows;
    if (r0 >= g.m) return;
    const int f = tile * kTile + lane;
    const int kw = (g.k + 31) >> 5, nw = (g.n + 31) >> 5;
    const uint32_t *zt = zb + (size_t)tile * nw * kTile + lane;
    uint32_t za[kSynKw];
#pragma unroll
    for (int w = 0; w < kSynKw; ++w) {
        uint32_t v = w < kw ? zt[w * kTile] : 0u;
        if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;  // A columns only
        za[w] = v;
    }
    uint32_t acc = 0u;
    for (int r = r0; r < min(r0 + kSynRows, g.m); ++r) {
        const uint32_t *ar = g.a_packed + (size_t)r * kw;
        const int q = g.k + r;  // identity column of row r
        uint32_t par = zt[(q >> 5) * kTile] >> (q & 31);
#pragma unroll
        for (int w = 0; w < kSynKw; ++w)
            if (w < kw) par += __builtin_popcount(ar[w] & za[w]);
        acc |= par & 1u;
    }
    if (acc) atomicOr(&bad[f], 1);
}

// The same row parities with lane = ROW (64 rows per wavefront), frame after
// frame: a few frames leave most lanes of syn_kernel idle (one frame: 1 of 64)
// and its 8-row chains set its time (~22 us); here a lane's A row is loaded
// once into registers and each frame's (z^1)_A words are wave-uniform.
constexpr int kSynRowFrames = 4;  // syn_row_kernel up to this many frames (one frame: 4.94 vs 5.30 ms; 8: 20.7 vs 20.0)
__global__ __launch_bounds__(256) void syn_row_kernel(DevGraph g, DevState st, const uint32_t *zb, int *bad) {
    const int tile = blockIdx.y;
    if (!st.tile_active[tile]) return;
    const int lane = threadIdx.x & 63;
    const int r = ((int)blockIdx.x * 4 + uniform(threadIdx.x >> 6)) * 64 + lane;  // this lane's row
    const int kw = (g.k + 31) >> 5, nw = (g.n + 31) >> 5;
    const bool row_ok = r < g.m;
    uint32_t ar[kSynKw];
#pragma unroll
    for (int w = 0; w < kSynKw; ++w) {
        uint32_t v = (row_ok && w < kw) ? g.a_packed[(size_t)r * kw + w] : 0u;
        if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;  // A columns only
        ar[w] = v;
    }
    const int q = g.k + (row_ok ? r : 0);  // identity column of row r
    unsigned long long live = __ballot(st.done[tile * kTile + lane] == 0);  // (lane as a frame index here)
    while (live != 0ull) {
        const int f = __ffsll((long long)live) - 1;  // uniform
        live &= live - 1ull;
        const uint32_t *zt = zb + (size_t)tile * nw * kTile + f;
        uint32_t par = zt[(q >> 5) * kTile] >> (q & 31);
#pragma unroll
        for (int w = 0; w < kSynKw; ++w)
            if (w < kw) par += __builtin_popcount(ar[w] & zt[w * kTile]);
        if (__ballot(row_ok && (par & 1u)) != 0ull && lane == 0) atomicOr(&bad[tile * kTile + f], 1);
    }
}

}  // namespace

int edge_max_deg() { return 64 * kEdgeKE; }

namespace {
int edge_slots(int deg) { return deg <= 256 ? 4 : deg <= 512 ? 8 : deg <= 768 ? 12 : 16; }
template <bool kFirst>
void cn_edge_launch(const DevGraph &g, const DevState &st, hipStream_t s) {
    const dim3 grid((unsigned)((g.m + 3) / 4), (unsigned)st.ntiles);
    switch (edge_slots(g.max_row_deg)) {
    case 4: cn_edge_kernel<kFirst, 4><<<grid, 256, 0, s>>>(g, st, kAtanhCoef); break;
    case 8: cn_edge_kernel<kFirst, 8><<<grid, 256, 0, s>>>(g, st, kAtanhCoef); break;
    case 12: cn_edge_kernel<kFirst, 12><<<grid, 256, 0, s>>>(g, st, kAtanhCoef); break;
    default: cn_edge_kernel<kFirst, 16><<<grid, 256, 0, s>>>(g, st, kAtanhCoef); break;
    }
}
}  // namespace

hipError_t launch_cn_edge(const DevGraph &g, const DevState &st, int it, hipStream_t s) {
    if (g.max_row_deg > 64 * kEdgeKE) return hipErrorInvalidValue;
    if (it == 0)
        cn_edge_launch<true>(g, st, s);
    else
        cn_edge_launch<false>(g, st, s);
    return hipGetLastError();
}

hipError_t launch_vn_edge_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                 int *cnt, int *bad, hipStream_t s) {
    if (!g.a_packed || g.max_col_deg > 64 * kEdgeKE || ((g.k + 31) >> 5) > kSynKw) return hipErrorInvalidValue;
    const dim3 vg((unsigned)((g.n + 3) / 4), (unsigned)st.ntiles);
    const int nl = nllr ? 1 : 0, fi = it == 0 ? 1 : 0;
    switch (edge_slots(g.max_col_deg)) {
    case 4: vn_edge_kernel<4><<<vg, 256, 0, s>>>(g, st, nl, zb, cnt, fi); break;
    case 8: vn_edge_kernel<8><<<vg, 256, 0, s>>>(g, st, nl, zb, cnt, fi); break;
    case 12: vn_edge_kernel<12><<<vg, 256, 0, s>>>(g, st, nl, zb, cnt, fi); break;
    default: vn_edge_kernel<16><<<vg, 256, 0, s>>>(g, st, nl, zb, cnt, fi); break;
    }
    if (st.count <= kSynRowFrames) {
        const int waves = (g.m + 63) / 64;
        syn_row_kernel<<<dim3((unsigned)((waves + 3) / 4), (unsigned)st.ntiles), 256, 0, s>>>(g, st, zb, bad);
    } else {
        const int waves = (g.m + kSynRows - 1) / kSynRows;
        syn_kernel<<<dim3((unsigned)((waves + 3) / 4), (unsigned)st.ntiles), 256, 0, s>>>(g, st, zb, bad);
    }
    return launch_tail_exit_decode(g, st, it, last, nllr, zb, cnt, bad, s);
}

}  // namespace ldpc
