// cn_sub.hip -- the split path's check-node pass on 16-frame sub-tiles (gfx950).
//
// Reference: python_ldpc_app/spa_decoder.py:112-168 (the CN update) with the
// M update :260-268 fused in front, exactly as cn_kernel (spa_kernels.hip):
//   M = L[col] - E_old (iteration 0 / a fresh streaming frame: M = L = ch),
//   t = tanh(M/2) clipped, P = t_0 * t_1 * ... left to right in ascending
//   column order, E_new = 2 atanh(clip(P/t)) (or the product of the others
//   for |t| <= 1e-10: such rows go to cn_rare_kernel untouched).
//
// cn_kernel walks a row with one wavefront (lane = frame) and, having no room
// for ~600 t values per lane, evaluates tanh twice per edge (pass 1 for the
// product, pass 2 for the quotients; 127 VALU per wavefront-edge, VALU-issue
// bound in the streaming tail: profiles/r3o_tailpmc).  Here one workgroup of W
// wavefronts takes one (tile, 16-frame sub-tile, row): lane = j*16 + f (lane
// group j = 0..3, frame f), the row's edges split into W contiguous wavefront
// chunks and each chunk into 4 contiguous lane-group pieces of <= K edges
// (tile_sub.hip's mapping), so every t stays in registers and tanh runs once
// per edge.  The left-to-right product runs group by group inside a wavefront
// (v_permlane16/32_swap, slots past a piece hold 1.0: exact no-ops) and
// wavefront by wavefront through LDS (W barriers).  The stores are the
// algorithmic 8 B of E_new per edge.  Bit-identical to cn_kernel /
// cn_row_kernel (the same fp64 operations in the same order).
//
// Used where those are slow: the long rows of the 2304 codes on few tiles --
// the streaming tail and small split batches (ldpc_api.cpp, spa_kernels.hip
// launch_cn: LDPC_CN_SUB).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "cn_common.h"
#include "spa_device.h"
#include "spa_math.h"

namespace ldpc {
namespace {

constexpr int kCsQ = 4;   // lane groups per wavefront
constexpr int kCsF = 16;  // frames per workgroup (lane = group * 16 + frame)

__device__ __forceinline__ double cs_ld_e(const double *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void cs_st_e(double *p, double v) { __builtin_nontemporal_store(v, p); }

// value of lane group jj moved into group jj+1 (lane = group*16 + frame: group
// = DPP row) by gfx950's v_permlane16_swap / v_permlane32_swap
__device__ __forceinline__ uint32_t cs_p16(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t cs_p32(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
__device__ __forceinline__ double cs_group_up(double v, int jj) {
    const uint64_t u = dbits(v);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    if (jj == 1) {  // row 1 -> row 2: [x0 x1 x0 x1], then its odd rows
        lo = cs_p16(cs_p32(lo, 0), 1);
        hi = cs_p16(cs_p32(hi, 0), 1);
    } else {  // row 0 -> 1, row 2 -> 3
        lo = cs_p16(lo, 0);
        hi = cs_p16(hi, 0);
    }
    return dfrom(((uint64_t)hi << 32) | lo);
}

// W wavefronts, K slots per lane (rows of <= W*4*K edges), phase-1 loads in S
// stages of K/S slots; WPS = min wavefronts per SIMD (register cap).
template <bool kFirst, bool kStream, int W, int K, int S, int WPS>
__global__ __launch_bounds__(64 * W, WPS) void cn_sub_kernel(DevGraph g, DevState st, int it_parity,
                                                             const int *__restrict__ col_idx,
                                                             const int *__restrict__ row_ptr, AtanhCoef ac) {
    static_assert(K % S == 0, "stages must divide the slots");
    __shared__ MathLds mlds;
    __shared__ double chain[kCsF];  // running product handed from wavefront to wavefront, per frame
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    const int j = lane >> 4, f = lane & 15;
    // XCD-aware: blocks b and b+8 share an XCD, so every (row, sub-tile) of a
    // tile gets the same b%8 and the tile's posteriors stay in that XCD's L2
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int per_tile = g.m * kCsQ;
    const int tile = (slot / per_tile) * 8 + (b & 7);
    const int rs = slot % per_tile;
    const int row = rs >> 2, sub = rs & 3;
    if (tile >= st.ntiles || !st.tile_active[tile]) return;  // block-uniform, before the table staging
    const int l64 = sub * kCsF + f;  // this lane's frame in the tile
    const int fr = tile * kTile + l64;
    const bool live = st.done[fr] == 0;
    // a sub-tile whose 16 frames have all stopped (the streaming tail's
    // compacted tiles thin out as frames finish) has nothing to store
    if (!__syncthreads_or(live)) return;
    fill_math_lds(mlds);
    __syncthreads();
    const LdsTanh ttab{mlds.tanh};
    const LdsAtanh ltab{mlds.atanh};
    const int beg = row_ptr[row], end = row_ptr[row + 1];
    const int deg = end - beg;
    if (deg == 0) return;  // spa_decoder.py:115-122
    const bool fresh = kStream && st.fresh[fr] != 0;
    double *Et = st.E + e_base(g, tile, l64);
    const double *Lt = (kFirst ? st.ch : st.L) + (size_t)tile * g.n * kTile + l64;
    const int C = (deg + W - 1) / W;
    const int c0 = beg + wave * C;
    const int cnt = max(0, min(deg - wave * C, C));  // wave-uniform
    const int CS = (cnt + kCsQ - 1) / kCsQ;         // wave-uniform piece length
    const int nj = max(0, min(cnt - j * CS, CS));   // this lane group's edges
    const int e0 = c0 + j * CS;                     // its first edge
    const int elast = nj > 0 ? e0 + nj - 1 : (cnt > 0 ? c0 : beg);  // a valid edge to load for padded slots

    double t[K];
    bool tiny = false;
#pragma unroll
    for (int h = 0; h < S; ++h) {
        constexpr int H = K / S;
        if (h * H < CS) {  // wave-uniform: a stage with slots in the chunk
            int col[H];
            double eo[H];
#pragma unroll
            for (int q = 0; q < H; ++q) {
                const int e = min(e0 + h * H + q, elast);
                col[q] = col_idx[e];
                eo[q] = kFirst ? 0.0 : cs_ld_e(&Et[(size_t)e * g.ef]);
            }
#pragma unroll
            for (int q = 0; q < H; ++q) t[h * H + q] = Lt[(size_t)col[q] * kTile];
#pragma unroll
            for (int q = 0; q < H; ++q) {
                const int i = h * H + q;
                const double M = kFirst ? t[i] : t[i] - ((kStream && fresh) ? 0.0 : eo[q]);  // :85-90 / :260-268
                const double tv = cn_tanh(M, ttab);                                        // :138-146
                tiny |= live && i < nj && !(fabs(tv) > kTiny);
                t[i] = i < nj ? tv : 1.0;  // past the piece: an exact no-op in the product
            }
        } else {
#pragma unroll
            for (int q = 0; q < H; ++q) t[h * H + q] = 1.0;
        }
    }
    if (__syncthreads_or(tiny)) {  // rare: this sub-tile's frames of the row to cn_rare_kernel
        if (threadIdx.x == 0) {
            const int at = atomicAdd(&st.rare_count[it_parity], 1);
            st.rare_list[at] = (int)rare_code(tile * g.m + row, 1u << sub);
        }
        return;
    }
    // P = t_0 * t_1 * ... strictly left to right (:151-152): group by group in
    // a wavefront, wavefront by wavefront through `chain`
    for (int w = 0; w < W; ++w) {
        if (wave == w && cnt > 0) {
            double P = w == 0 ? 1.0 : chain[f];  // 1.0 * t0 == t0 exactly
#pragma unroll
            for (int jj = 0; jj < kCsQ; ++jj) {
#pragma unroll
                for (int i = 0; i < K; ++i) P = P * t[i];
                if (jj + 1 < kCsQ) P = cs_group_up(P, jj);
            }
            if (j == kCsQ - 1) chain[f] = P;
        }
        __syncthreads();
    }
    if (cnt == 0) return;
    const double P = chain[f];
    // q = P/t (div_nr where exact, cn_common.h); E_new = 2 atanh(clip(q)), or
    // 2q when every quotient of the wavefront is below 2^-27 (spa_math.h
    // kAtanhIdent), slot by slot; frame-less lanes do not vote.
    // Saturated rows (the streaming tail at 2.5-3 dB: the frames that fail
    // there have 85-97 % of their t at +-CL) give most slots of a lane one
    // quotient magnitude: a slot where every live lane's |q| equals its slot-0
    // |q| takes slot 0's E_new with its own sign -- atanh_f(clip_cl(q)) is odd
    // bit for bit and 2q trivially so (tests/test_math.py), so this is the
    // same value, one atanh per lane and row instead of one per slot
    // (tile8.hip's memo).  Lanes that do not vote keep values nothing stores.
    const double lim = live ? kAtanhIdent : INFINITY;
    double key = 0.0, E0 = 0.0;
    auto en = [&](int i, double q) {
        double En;
        if (__ballot(!(fabs(q) < lim)) == 0ull)
            En = 2.0 * q;
        else if (i > 0 && __ballot(live && i < nj && fabs(q) != key) == 0ull)
            En = dfrom((dbits(E0) & 0x7fffffffffffffffull) | (dbits(q) & 0x8000000000000000ull));
        else
            En = 2.0 * atanh_f(clip_cl(q), ltab, ac);
        if (i == 0) {
            key = fabs(q);
            E0 = En;
        }
        return En;
    };
    if (div_nr_ok(live ? P : 1.0)) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if (i < CS) {  // wave-uniform
                const double En = en(i, div_nr(P, t[i]));
                if (live && i < nj) cs_st_e(&Et[(size_t)(e0 + i) * g.ef], En);
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (i < CS) {
            const double En = en(i, P / t[i]);
            if (live && i < nj) cs_st_e(&Et[(size_t)(e0 + i) * g.ef], En);
        }
    }
}

}  // namespace

// The shapes: rows <= 8*4*20 = 640 edges (wimax_2304_0.5: 416-632) in 8
// wavefronts x 20 slots, phase-1 loads in 4 stages, >= 6 wavefronts per SIMD;
// rows <= 8*4*30 = 960 (the r3/4 codes: <= 931) in 8 x 30.  Measured and not
// kept (profiles/r4b_ab, r4c_ab): 16 x 10 and 16 x 15 shapes, indices
// requested up front, other stage counts.
int cn_sub_shape(const DevGraph &g) {
    if (g.max_row_deg <= 8 * kCsQ * 20) return 20;
    if (g.max_row_deg <= 8 * kCsQ * 30) return 30;
    return 0;
}

template <bool kFirst, bool kStream>
static hipError_t launch_cn_sub_t(const DevGraph &g, const DevState &st, int par, hipStream_t s) {
    const unsigned grid = (unsigned)(((st.ntiles + 7) / 8) * 8 * g.m * kCsQ);
    const int *ci = g.col_idx, *rp = g.row_ptr;
    switch (cn_sub_shape(g)) {
        case 20:
            cn_sub_kernel<kFirst, kStream, 8, 20, 4, 6><<<grid, 64 * 8, 0, s>>>(g, st, par, ci, rp, kAtanhCoef);
            break;
        case 30:
            cn_sub_kernel<kFirst, kStream, 8, 30, 6, 4><<<grid, 64 * 8, 0, s>>>(g, st, par, ci, rp, kAtanhCoef);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_cn_sub(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream) {
    const int par = it & 1;
    if (stream) return launch_cn_sub_t<false, true>(g, st, par, s);
    if (it == 0) return launch_cn_sub_t<true, false>(g, st, par, s);
    return launch_cn_sub_t<false, false>(g, st, par, s);
}

}  // namespace ldpc
