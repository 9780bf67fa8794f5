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

}  // namespace ldpc
