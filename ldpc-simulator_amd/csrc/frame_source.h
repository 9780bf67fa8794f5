// frame_source.h -- the on-device synthetic frame source's random draws,
// shared by every generator (spa_kernels.hip: H_std = [A|I] codes;
// ira_kernels.hip: IRA codes) so a frame index always yields the same info
// bits and the same noise.  CPU restatement: oracle/channel_oracle.c.
//   info word w of frame F, SNR point p: Philox4x32-10 key (seed), counter
//     {F lo, F hi, w/4, p<<1}, word w%4 of the output
//   noise of columns 2b, 2b+1: counter {F lo, F hi, b, (p<<1)|1}, two 52-bit
//     uniforms, Box-Muller r*cos / r*sin
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "spa_device.h"

namespace ldpc {

__device__ __forceinline__ double u52(uint32_t hi, uint32_t lo) {
    const uint64_t x = (((uint64_t)hi << 32) | lo) >> 12;  // 52 random bits
    return ((double)x + 0.5) * 0x1p-52;                    // exact, in (0,1)
}

// Info words 4*blk .. 4*blk+3 of frame F.
__device__ __forceinline__ void info_block(uint64_t seed, int64_t F, int snr_point, int blk, uint32_t out[4]) {
    out[0] = (uint32_t)F;
    out[1] = (uint32_t)((uint64_t)F >> 32);
    out[2] = (uint32_t)blk;
    out[3] = (uint32_t)snr_point << 1;
    philox4x32_10(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// N(0,1) pair for columns 2*b and 2*b+1 of frame F.
__device__ __forceinline__ void noise_pair(uint64_t seed, int64_t F, int snr_point, int b, double g[2]) {
    uint32_t c[4] = {(uint32_t)F, (uint32_t)((uint64_t)F >> 32), (uint32_t)b, ((uint32_t)snr_point << 1) | 1u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u1 = u52(c[0], c[1]);
    const double u2 = u52(c[2], c[3]);
    const double r = sqrt(-2.0 * log(u1));
    // cos/sin(2 pi u2) as sincospi(2 u2): no Payne-Hanek reduction; 2 u2 is
    // exact, and the result differs from sin/cos(fl(2 pi u2)) (the CPU
    // restatement) by ~1e-16 relative
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    g[0] = r * cs;
    g[1] = r * sn;
}

// BPSK bit0 -> -1, bit1 -> +1 (channel.py:49); y = x + sigma^2 g (noise std is
// sigma^2, channel.py:68-76); llr = 2y/sigma^2 (channel.py:80).
__device__ __forceinline__ double channel_llr(uint32_t bit, double g, double s2) {
    const double x = bit ? 1.0 : -1.0;
    const double y = x + s2 * g;
    return (2.0 * y) / s2;
}

// Test-only erasures (LDPC_F_TEST_ZERO; tests/test_gpu_rare_stream.py): with
// g.zinj != 0, frames F with F % 4 == 1 get a channel LLR of exactly 0.0 on
// identity column k + (131 F + 7) mod m and on information column
// (37 F + 3) mod k.  An identity column has degree 1 in H_std = [A | I], so
// its M = L - E = (0 + E) - E is exactly 0 on EVERY iteration: the row takes
// the reference's |t| <= 1e-10 branch (spa_decoder.py:159-164) on each pass
// the frame makes -- in the streaming kernels and, for frames still running
// at hand-off, in the split tail (cn_sub_kernel -> cn_rare_kernel).  The
// information column does the same on the frame's first pass.  The predicate
// is restated in the test, which checks the generator against it.
__device__ __forceinline__ bool test_zero_llr(const DevGraph &g, long long F, int j) {
    if (!g.zinj || (F & 3) != 1) return false;
    const unsigned long long u = (unsigned long long)F;
    return j == g.k + (int)((131ull * u + 7ull) % (unsigned long long)g.m) ||
           (g.k > 0 && j == (int)((37ull * u + 3ull) % (unsigned long long)g.k));
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------ cooperative slot refill
// Streaming refill by the WHOLE workgroup, with generate_kernel's draws
// (frame_kernels.hip: the same frames bit for bit): slot f (0..F-1, tile lane lane0 + f) takes frame
// gidx[f], or nothing when gidx[f] < 0.  ustage: LDS [kw][F] words, zero on
// return (a refilled slot's words are written before they are read; the
// caller puts a barrier after).  Thread
// t = worker * F + f: first the info words as (Philox block, slot) tasks,
// then column pairs worker, worker + nworkers, ... of every refilled slot --
// all wavefronts share the n/2 noise draws and m parity rows of a frame that
// one wavefront generated alone before (a 2304-bit frame: ~40 % of a pass of
// the streaming sub-tile decoder at 3 dB, where most slots refill every pass).
// Every thread of the block calls it (it holds two barriers).
template <int F>
__device__ inline void gen_slots(const DevGraph &g, const DevState &st, int tile, int lane0, const long long *gidx,
                                 uint32_t *ustage, uint64_t seed, int snr_point, double sigma) {
    const int kw = (g.k + 31) >> 5;
    const int nthr = blockDim.x;
    // info bits: data_buffer.py:23 / generator.py:7-9
    for (int t = threadIdx.x; t < ((kw + 3) >> 2) * F; t += nthr) {
        const int f = t % F, blk = t / F;
        const long long Fi = gidx[f];
        if (Fi < 0) continue;
        uint32_t c[4];
        info_block(seed, Fi, snr_point, blk, c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int w = blk * 4 + q;
            if (w >= kw) break;
            uint32_t v = c[q];
            if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;
            ustage[w * F + f] = v;
            st.ubits[((size_t)tile * kw + w) * kTile + lane0 + f] = v;
        }
    }
    __syncthreads();
    // codeword [u, A.u mod 2] + BPSK + AWGN (channel.py:49,68-80), L = ch
    const int f = threadIdx.x % F, worker = threadIdx.x / F, nwork = nthr / F;
    const long long Fi = gidx[f];
    if (Fi >= 0) {
        const double s2 = sigma * sigma;
        double *Ct = st.ch + (size_t)tile * g.n * kTile + lane0 + f;
        double *Lt = st.L + (size_t)tile * g.n * kTile + lane0 + f;
        for (int b = worker; 2 * b < g.n; b += nwork) {
            double gz[2];
            noise_pair(seed, Fi, snr_point, b, gz);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = 2 * b + q;
                if (j >= g.n) break;
                uint32_t bit;
                if (j < g.k) {
                    bit = (ustage[(j >> 5) * F + f] >> (j & 31)) & 1u;
                } else {  // parity(A_row & u), A bit-packed
                    const uint32_t *ar = g.a_packed + (size_t)(j - g.k) * kw;
                    uint32_t acc = 0u;
                    for (int w = 0; w < kw; ++w) acc ^= ar[w] & ustage[w * F + f];
                    bit = (uint32_t)__popc(acc) & 1u;
                }
                const double llr = test_zero_llr(g, Fi, j) ? 0.0 : channel_llr(bit, gz[q], s2);
                Ct[(size_t)j * kTile] = llr;
                Lt[(size_t)j * kTile] = llr;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kw * F; i += nthr) ustage[i] = 0u;
}

}  // namespace ldpc
