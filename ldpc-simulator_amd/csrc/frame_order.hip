// frame_order.hip -- supply order of a streamed Monte-Carlo point (gfx950).
//
// The streaming schedule (ldpc_api.cpp mc_stream_point) decodes a point's
// frames through a fixed set of slots; a slot takes the next frame as soon as
// its own stops.  Every frame decodes exactly as in the static schedule, so
// the counters (main.py:130-138, sums over the point's frames) do not depend
// on the ORDER in which frames enter the slots -- but the wall time does: a
// frame that fails runs all max_iter iterations, and one that enters late
// keeps the step going long after the supply is out (the streaming tail: at
// 3 dB on wimax_2304_0.5, ~1,150 failing frames running ~44 more iterations
// on a few tiles, ~290 of a ~530 ms step).  Longest job first:
// the frames are ranked by what a receiver sees before decoding -- the number
// of unsatisfied checks of the channel's hard decisions (syndrome weight of
// H_std (llr > 0)) -- and supplied heaviest first, so the frames that will
// run long start while the slots are still being refilled.
//
// Round 5: equal syndrome weights (most frames have none at 2.5-3 dB) are
// ranked by the channel reliability of the weakest identity bit whose single
// check row has odd degree, least reliable first, on graphs where at most
// half the rows have odd degree (wimax_2304_0.5).  There the frames that fail
// with error-free or one-error hard decisions are exactly those (the
// reference's check rule returns a wrong-sign extrinsic on odd-degree rows,
// SURVEY.md §0.3, which flips a weak degree-1 bit): on 8,000 oracle-decoded
// frames at 3 dB all 18 zero-syndrome failures rank in the first 1.3 % of the
// zero-syndrome frames (index order: spread to 85 %), so the last failing
// frame starts in the first ~9 % of the supply instead of at its end.
// Codes with mostly odd rows (the r3/4 codes: there the most reliable frames
// fail) keep index order within a syndrome weight.
//
// frame_score_kernel regenerates each frame with the device frame source's
// own draws (frame_source.h: info_block / noise_pair / channel_llr, the same
// bits gen_slots writes into the slots later) and counts its unsatisfied
// rows (and that weakest |llr|); hipcub's stable radix sort orders the local
// frame indices by descending key = weight << 16 | reliability rank (ties in
// index order: deterministic).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "frame_source.h"
#include "spa_device.h"

namespace ldpc {
namespace {

constexpr int kScoreThreads = 256;

__global__ __launch_bounds__(kScoreThreads) void frame_score_kernel(DevGraph g, uint64_t seed, int snr_point,
                                                                    double sigma, int64_t frame0, int total,
                                                                    uint32_t *score, int *idx) {
    extern __shared__ uint32_t sh[];  // u [kw] | hard bits [nw]
    __shared__ uint32_t wsum[kScoreThreads / 64];
    __shared__ float wmin[kScoreThreads / 64];
    const int kw = (g.k + 31) >> 5, nw = (g.n + 31) >> 5;
    uint32_t *u = sh, *hb = sh + kw;
    const double s2 = sigma * sigma;
    const uint32_t klast = (g.k & 31) ? (1u << (g.k & 31)) - 1u : ~0u;  // A columns of hard-bit word kw-1
    for (int f = blockIdx.x; f < total; f += gridDim.x) {
        const int64_t F = frame0 + f;
        // info bits (data_buffer.py:23; gen_slots' draws)
        for (int t = threadIdx.x; t < ((kw + 3) >> 2); t += blockDim.x) {
            uint32_t c[4];
            info_block(seed, F, snr_point, t, c);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int w = t * 4 + q;
                if (w >= kw) break;
                u[w] = (w == kw - 1) ? (c[q] & klast) : c[q];
            }
        }
        for (int i = threadIdx.x; i < nw; i += blockDim.x) hb[i] = 0u;
        __syncthreads();
        // codeword [u, A.u], BPSK + AWGN, LLR (channel.py:49,68-80); hard bit = llr > 0
        float weak = INFINITY;  // min |llr| over identity bits of odd-degree rows
        for (int b = threadIdx.x; 2 * b < g.n; b += blockDim.x) {
            double gz[2];
            noise_pair(seed, F, snr_point, b, gz);
            uint32_t hv = 0u;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = 2 * b + q;
                if (j >= g.n) break;
                uint32_t bit;
                if (j < g.k) {
                    bit = (u[j >> 5] >> (j & 31)) & 1u;
                } else {
                    const uint32_t *ar = g.a_packed + (size_t)(j - g.k) * kw;
                    uint32_t acc = 0u;
                    for (int w = 0; w < kw; ++w) acc ^= ar[w] & u[w];
                    bit = (uint32_t)__popc(acc) & 1u;
                }
                const double l = test_zero_llr(g, F, j) ? 0.0 : channel_llr(bit, gz[q], s2);
                if (l > 0.0) hv |= 1u << q;
                if (g.lpt_weak_id && j >= g.k && ((g.row_ptr[j - g.k + 1] - g.row_ptr[j - g.k]) & 1))
                    weak = fminf(weak, (float)fabs(l));
            }
            if (hv) atomicOr(&hb[(2 * b) >> 5], hv << ((2 * b) & 31));
        }
        __syncthreads();
        // unsatisfied rows of H_std = [A | I_m] on the hard decisions
        uint32_t cnt = 0u;
        for (int r = threadIdx.x; r < g.m; r += blockDim.x) {
            const uint32_t *ar = g.a_packed + (size_t)r * kw;
            uint32_t par = hb[(g.k + r) >> 5] >> ((g.k + r) & 31);
            for (int w = 0; w < kw; ++w) par += __popc(ar[w] & (w == kw - 1 ? hb[w] & klast : hb[w]));
            cnt += par & 1u;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cnt += __shfl_xor(cnt, o);
            weak = fminf(weak, __shfl_xor(weak, o));
        }
        if ((threadIdx.x & 63) == 0) {
            wsum[threadIdx.x >> 6] = cnt;
            wmin[threadIdx.x >> 6] = weak;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t s = 0u;
            float w = INFINITY;
#pragma unroll
            for (int i = 0; i < kScoreThreads / 64; ++i) {
                s += wsum[i];
                w = fminf(w, wmin[i]);
            }
            // |llr| >= 0: its float bits rise with it; the top 16 of 31, inverted
            const uint32_t rel = g.lpt_weak_id ? 0xffffu - (__float_as_uint(w) >> 15) : 0u;
            // the weight saturates at 16 bits (launch_frame_order also rejects m > 65535)
            score[f] = (min(s, 0xffffu) << 16) | rel;
            idx[f] = f;
        }
        __syncthreads();  // u / hb / wsum are rewritten by the next frame
    }
}

}  // namespace

// Temporary bytes the sort needs for `total` frames.
size_t frame_order_temp_bytes(int total) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                       (const int *)nullptr, (int *)nullptr, total, 0, 32);
    return bytes;
}

// order[0..total) = the point's local frame indices, heaviest syndrome first
// (equal weights: least reliable odd-row identity bit first, lpt_weak_id).
// keys: 2 x total uint32, vals: total int scratch, temp: frame_order_temp_bytes.
hipError_t launch_frame_order(const DevGraph &g, uint64_t seed, int snr_point, double sigma, int64_t frame0,
                              int total, uint32_t *keys, int *vals, int *order, void *temp, size_t temp_bytes,
                              hipStream_t s) {
    if (total <= 0) return hipSuccess;
    if (!g.std_form || !g.a_packed || g.m > 65535) return hipErrorInvalidValue;
    const int kw = (g.k + 31) >> 5, nw = (g.n + 31) >> 5;
    const int grid = total < 8192 ? total : 8192;
    frame_score_kernel<<<grid, kScoreThreads, (size_t)(kw + nw) * sizeof(uint32_t), s>>>(g, seed, snr_point, sigma,
                                                                                         frame0, total, keys, vals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t bytes = temp_bytes;
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, bytes, keys, keys + total, vals, order, total, 0, 32, s);
}

}  // namespace ldpc
