// frame_kernels.hip -- the on-device synthetic frame source,
// gfx950.  Replaces DataBuffer(k) + encode + Channel mode 1 of the reference
// (data_buffer.py:16-82, channel.py:38-81, generator.py:7-9); random draws in
// frame_source.h, CPU restatement oracle/channel_oracle.c.
//
// Frames are generated column-parallel, tile layout (lane = frame):
//   frame_ubits     info words u (Philox blocks of 4 words)
//   std_parity      H_std = [A | I]: parity word of 32 rows, p_r = parity(A_r & u)
//                   (A bit-packed per row, uniform loads) -- one wavefront per word
//   ira_sbits       IRA H = [H_info | staircase]: s_r = parity of row r's info bits,
//   ira_carry       stored as in-word prefix XOR + exclusive scan of the word
//                   parities: p_r = p_{r-1} ^ s_r, the accumulator
//   frame_channel   bit -> BPSK -> + sigma^2 N(0,1) -> llr = 2y/sigma^2, written as
//                   fp64 ch (parity decoder, LDS physical decoder, export) or as
//                   the tile physical decoder's fp32 Lambda = L = -llr
// Every kernel has >= ntiles x (n/128 or m/128) wavefronts, so even a small
// chunk fills the chip (the streaming refill, where single slots are
// regenerated, uses frame_source.h's gen_slots: the same draws).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "frame_source.h"
#include "spa_device.h"

namespace ldpc {
namespace {

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// bit i of the result = XOR of bits 0..i of x
__device__ __forceinline__ uint32_t prefix_xor(uint32_t x) {
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    return x;
}

__global__ __launch_bounds__(64) void frame_ubits_kernel(DevGraph g, DevState st, uint64_t seed, int snr_point,
                                                       int64_t frame0, int blk_per_block) {
    const int kw = (g.k + 31) >> 5;
    const int nblk = (kw + 3) >> 2;
    const int nbc = (nblk + blk_per_block - 1) / blk_per_block;
    const int tile = blockIdx.x / nbc, bc = blockIdx.x % nbc;
    const int lane = threadIdx.x;
    const int64_t F = frame0 + tile * kTile + lane;
    const int b1 = min(nblk, (bc + 1) * blk_per_block);
    for (int blk = bc * blk_per_block; blk < b1; ++blk) {
        uint32_t c[4];
        info_block(seed, F, snr_point, blk, c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int w = blk * 4 + q;
            if (w >= kw) break;
            uint32_t v = c[q];
            if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;
            st.ubits[((size_t)tile * kw + w) * kTile + lane] = v;
        }
    }
}

// s_r = parity of row r's info bits; one wavefront -> 32 rows -> one word,
// stored as its in-word prefix XOR; the word's total parity (bit 31 of the
// prefix) is packed into wpar for the carry scan.
__global__ __launch_bounds__(256) void ira_sbits_kernel(DevGraph g, DevState st, PhysTile pt,
                                                        const int *__restrict__ row_ptr,
                                                        const int *__restrict__ col_idx) {
    const int kw = (g.k + 31) >> 5;
    const int mw = (g.m + 31) >> 5;
    const int per_tile = (mw + 3) >> 2;
    const int tile = blockIdx.x / per_tile;
    const int w = (blockIdx.x % per_tile) * 4 + uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= mw) return;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
    uint32_t word = 0u;
    const int r1 = min(g.m, (w + 1) * 32);
    for (int r = w * 32; r < r1; ++r) {
        uint32_t b = 0u;
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
            const int c = col_idx[e];
            if (c < g.k) b ^= Ut[(c >> 5) * kTile] >> (c & 31);
        }
        word |= (b & 1u) << (r & 31);
    }
    const uint32_t x = prefix_xor(word);
    pt.pbits[((size_t)tile * mw + w) * kTile + lane] = x;
    const int mw32 = (mw + 31) >> 5;
    if (x >> 31) atomicOr(&pt.wpar[((size_t)tile * mw32 + (w >> 5)) * kTile + lane], 1u << (w & 31));
}

// wpar bit w := parity of all s words before word w (exclusive scan), so
// p_r = bit (r%32) of pbits[r/32] ^ wpar bit (r/32): the staircase accumulator.
__global__ __launch_bounds__(64) void ira_carry_kernel(DevGraph g, PhysTile pt) {
    const int mw32 = (((g.m + 31) >> 5) + 31) >> 5;
    const int tile = blockIdx.x, lane = threadIdx.x;
    uint32_t *Wt = pt.wpar + (size_t)tile * mw32 * kTile + lane;
    uint32_t carry = 0u;
    for (int W = 0; W < mw32; ++W) {
        const uint32_t z = prefix_xor(Wt[W * kTile]);
        Wt[W * kTile] = (z << 1) ^ (0u - carry);
        carry ^= z >> 31;
    }
}

// to_lambda: write the tile decoder's fp32 Lambda = L = -llr directly
// (kFramesTileLambda), else the fp64 channel LLRs ch (kFramesCh).
__global__ __launch_bounds__(64) void frame_channel_kernel(DevGraph g, DevState st, PhysTile pt, uint64_t seed,
                                                         int snr_point, double sigma, int64_t frame0,
                                                         int to_lambda) {
    const int kw = (g.k + 31) >> 5;
    const int mw = (g.m + 31) >> 5;
    const int npairs = (g.n + 1) >> 1;
    const int per_tile = (npairs + 63) >> 6;
    const int tile = blockIdx.x / per_tile;
    const int b0 = (blockIdx.x % per_tile) * 64;
    const int lane = threadIdx.x;
    const int f = tile * kTile + lane;
    const bool valid = f < st.count;
    const int64_t F = frame0 + f;
    const double s2 = sigma * sigma;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
    const int mw32 = (mw + 31) >> 5;
    const uint32_t *Pt = pt.pbits + (size_t)tile * mw * kTile + lane;
    const uint32_t *Wt = pt.wpar + (size_t)tile * mw32 * kTile + lane;
    double *Ct = st.ch + (size_t)tile * g.n * kTile + lane;
    float *Lamt = pt.Lam + (size_t)tile * g.n * kTile + lane;
    float *Lt = pt.L + (size_t)tile * g.n * kTile + lane;
    const int b1 = min(npairs, b0 + 64);
    for (int b = b0; b < b1; ++b) {
        double gz[2];
        noise_pair(seed, F, snr_point, b, gz);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = 2 * b + q;
            if (j >= g.n) break;
            const int r = j - g.k;
            const int w = r >> 5;
            const uint32_t bit = j < g.k ? (Ut[(j >> 5) * kTile] >> (j & 31)) & 1u
                                         : ((Pt[w * kTile] >> (r & 31)) ^ (Wt[(w >> 5) * kTile] >> (w & 31))) & 1u;
            const double llr = valid && !test_zero_llr(g, F, j) ? channel_llr(bit, gz[q], s2) : 0.0;
            if (to_lambda) {
                Lamt[j * kTile] = -(float)llr;
                Lt[j * kTile] = -(float)llr;
            } else {
                Ct[j * kTile] = llr;
            }
        }
    }
}


// The same draws written row-major, Lambda = -llr as fp32 [count][n] (the LDS
// physical decoder reads a frame contiguously): one wavefront per (frame, 64
// column pairs), lane = column pair.
__global__ __launch_bounds__(64) void frame_channel_row_kernel(DevGraph g, DevState st, PhysTile pt, uint64_t seed,
                                                             int snr_point, double sigma, int64_t frame0,
                                                             float *__restrict__ row_out) {
    const int kw = (g.k + 31) >> 5;
    const int mw = (g.m + 31) >> 5;
    const int mw32 = (mw + 31) >> 5;
    const int npairs = (g.n + 1) >> 1;
    const int per_frame = (npairs + 63) >> 6;
    const int f = blockIdx.x / per_frame;
    const int b = (blockIdx.x % per_frame) * 64 + threadIdx.x;
    if (f >= st.count || b >= npairs) return;
    const int tile = f >> 6, lf = f & 63;
    const double s2 = sigma * sigma;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lf;
    const uint32_t *Pt = pt.pbits + (size_t)tile * mw * kTile + lf;
    const uint32_t *Wt = pt.wpar + (size_t)tile * mw32 * kTile + lf;
    double gz[2];
    noise_pair(seed, frame0 + f, snr_point, b, gz);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int j = 2 * b + q;
        if (j >= g.n) break;
        const int r = j - g.k;
        const int w = r >> 5;
        const uint32_t bit = j < g.k ? (Ut[(j >> 5) * kTile] >> (j & 31)) & 1u
                                     : ((Pt[w * kTile] >> (r & 31)) ^ (Wt[(w >> 5) * kTile] >> (w & 31))) & 1u;
        row_out[(size_t)f * g.n + j] = test_zero_llr(g, frame0 + f, j) ? -0.0f : -(float)channel_llr(bit, gz[q], s2);
    }
}

// p_r = parity(A_r & u) for the 32 rows of one word; wpar stays zero (no carry).
// KW > 0: the frame's u words are held in registers (kw <= KW) and A's words
// come through scalar loads; KW = 0: any kw, u re-read per row.
template <int KW>
__global__ __launch_bounds__(256) void std_parity_kernel(DevGraph g, DevState st, PhysTile pt,
                                                         const uint32_t *__restrict__ apack) {
    const int kw = (g.k + 31) >> 5;
    const int mw = (g.m + 31) >> 5;
    const int per_tile = (mw + 3) >> 2;
    const int tile = blockIdx.x / per_tile;
    const int w = (blockIdx.x % per_tile) * 4 + uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= mw) return;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
    uint32_t word = 0u;
    const int r1 = min(g.m, (w + 1) * 32);
    if constexpr (KW > 0) {
        uint32_t u[KW];
#pragma unroll
        for (int i = 0; i < KW; ++i) u[i] = i < kw ? Ut[i * kTile] : 0u;
        for (int r = w * 32; r < r1; ++r) {
            const uint32_t *ar = apack + (size_t)r * kw;
            uint32_t acc = 0u;
#pragma unroll
            for (int i = 0; i < KW; ++i)
                if (i < kw) acc ^= ar[i] & u[i];
            word |= ((uint32_t)__popc(acc) & 1u) << (r & 31);
        }
    } else {
        for (int r = w * 32; r < r1; ++r) {
            const uint32_t *ar = apack + (size_t)r * kw;
            uint32_t acc = 0u;
            for (int i = 0; i < kw; ++i) acc ^= ar[i] & Ut[i * kTile];
            word |= ((uint32_t)__popc(acc) & 1u) << (r & 31);
        }
    }
    pt.pbits[((size_t)tile * mw + w) * kTile + lane] = word;
}

}  // namespace

hipError_t launch_frames(const DevGraph &g, const DevState &st, const PhysTile &pt, uint64_t seed, int snr_point,
                         double sigma, int64_t frame0, FramesOut out, float *row_out, hipStream_t s) {
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int nblk = (kw + 3) >> 2, bpb = 16;
    const int nbc = (nblk + bpb - 1) / bpb;
    const int mw32 = (mw + 31) >> 5;
    hipError_t e = hipMemsetAsync(pt.wpar, 0, sizeof(uint32_t) * (size_t)st.ntiles * mw32 * kTile, s);
    if (e != hipSuccess) return e;
    if (g.k > 0) frame_ubits_kernel<<<st.ntiles * nbc, 64, 0, s>>>(g, st, seed, snr_point, frame0, bpb);
    if (g.ira) {
        ira_sbits_kernel<<<st.ntiles * ((mw + 3) >> 2), 256, 0, s>>>(g, st, pt, g.row_ptr, g.col_idx);
        ira_carry_kernel<<<st.ntiles, 64, 0, s>>>(g, pt);
    } else {
        const unsigned grid = (unsigned)(st.ntiles * ((mw + 3) >> 2));
        if (kw <= 16)
            std_parity_kernel<16><<<grid, 256, 0, s>>>(g, st, pt, g.a_packed);
        else if (kw <= 64)
            std_parity_kernel<64><<<grid, 256, 0, s>>>(g, st, pt, g.a_packed);
        else
            std_parity_kernel<0><<<grid, 256, 0, s>>>(g, st, pt, g.a_packed);
    }
    const int npairs = (g.n + 1) >> 1;
    if (out == kFramesRowLambda)
        frame_channel_row_kernel<<<st.count * ((npairs + 63) >> 6), 64, 0, s>>>(g, st, pt, seed, snr_point, sigma,
                                                                              frame0, row_out);
    else
        frame_channel_kernel<<<st.ntiles * ((npairs + 63) >> 6), 64, 0, s>>>(
            g, st, pt, seed, snr_point, sigma, frame0, out == kFramesTileLambda ? 1 : 0);
    return hipGetLastError();
}

}  // namespace ldpc
