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


__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------ per-lane frame generation
// (streaming refill; whole chunks use frame_kernels.hip).  u bits live in LDS
// ([kw][64], each lane reads only its own column, so no barrier is needed).
// Frame F of SNR point `snr_point` into lane `lane` of `tile`: info bits (ubits
// and the lane's LDS column `ul`), channel LLRs ch[tile][j][lane].  With
// `set_L`, also L = ch (a streaming refill: the next CN then forms M = L - 0).
__device__ inline void gen_lane(const DevGraph &g, const DevState &st, int tile, int lane, int64_t F, uint64_t seed,
                         int snr_point, double sigma, const uint32_t *__restrict__ apack, uint32_t *ul, bool valid,
                         bool set_L) {
    const int kw = (g.k + 31) >> 5;
    // info bits: data_buffer.py:23 / generator.py:7-9 (random.randint(0,1) per bit)
    for (int blk = 0; blk * 4 < kw; ++blk) {
        uint32_t c[4];
        info_block(seed, F, snr_point, blk, c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int w = blk * 4 + q;
            if (w >= kw) break;
            uint32_t v = c[q];
            if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;
            ul[w * kTile + lane] = v;
            st.ubits[((size_t)tile * kw + w) * kTile + lane] = v;
        }
    }
    // codeword [u, A.u mod 2] + BPSK + AWGN (channel.py:49,68-80)
    const double s2 = sigma * sigma;
    double *Ct = st.ch + (size_t)tile * g.n * kTile + lane;
    double *Lt = st.L + (size_t)tile * g.n * kTile + lane;
    for (int jb = 0; jb < g.n; jb += 2) {
        double gz[2];
        noise_pair(seed, F, snr_point, jb >> 1, gz);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = jb + q;
            if (j >= g.n) break;
            uint32_t bit;
            if (j < g.k) {
                bit = (ul[(j >> 5) * kTile + lane] >> (j & 31)) & 1u;
            } else {  // parity bit of row j-k = parity(A_row & u), A bit-packed (uniform loads)
                const uint32_t *ar = apack + (size_t)(j - g.k) * kw;
                uint32_t acc = 0u;
                for (int w = 0; w < kw; ++w) acc ^= ar[w] & ul[w * kTile + lane];
                bit = (uint32_t)__popc(acc) & 1u;
            }
            const double llr = valid ? channel_llr(bit, gz[q], s2) : 0.0;
            Ct[j * kTile] = llr;
            if (set_L) Lt[j * kTile] = llr;
        }
    }
}

}  // namespace ldpc
