// phys_tile.hip -- physical mode with the decoder state in HBM (SURVEY.md
// §8 f4, BASELINE config 5), gfx950.
//
// Same arithmetic as phys_kernels.hip (phys_math.h, identical operation
// order, so both paths give bit-identical results), for codes whose per-frame
// state does not fit in LDS (DVB-S2-profile n=64800: E 0.9 MB + L 0.26 MB per
// frame).  Layout as the parity decoder: 64 frames per tile, lane = frame,
//   E32 [tile][nnz][64] fp32   L32 [tile][n][64] fp32   ch [tile][n][64] fp64
// so every load/store of a wavefront is 256 B contiguous.
//
//   phys_cn_tile  one wavefront per (tile, 4 check rows): per row, gather
//                 L[col] and E_old, keep phi(|M|) and the signs of M in
//                 registers (rows of degree <= kDeg), write E_new: 12 B/edge.
//                 The same sweep forms the row parity of the hard decisions
//                 (L < 0) -> bad[it&1][frame]: the syndrome of the previous
//                 iteration's posterior, for free.
//   phys_vn_tile  one wavefront per (tile, 8 columns): L = Lambda + sum E
//                 (Lambda = -channel LLR) in CSC order: 4 B/edge + 12 B/col.
//                 A frame whose syndrome was zero stops here, converged at
//                 the previous iteration (exactly the LDS kernel's exit).
// After the last iteration a syndrome-only CN sweep and phys_tile_final give
// the frames that converge on it.
// Monte-Carlo runs (counters only) compact: once at most a quarter of the
// launched slots still run, the finished frames are counted and the running
// ones move into the first tiles (phys_compact_*), so the last sweeps launch
// those tiles only -- at 1 dB on the DVB-S2 profile the fourth CN sweep ran
// for ~5 % of the frames, scattered over every tile, at the cost of a full
// sweep (profiles/r5s_c5).  done[]: 0 running, 1 finished (to be counted),
// 2 counted, moved away, or no frame.  Each (tile, row block) and (tile, column
// block) is placed XCD-aware like cn_kernel.
// Frames come from frame_kernels.hip (directly as fp32 Lambda/L for IRA
// codes, else as fp64 ch converted by phys_tile_init).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "phys_math.h"
#include "spa_device.h"

namespace ldpc {
namespace {

// The fp32 message array (streamed once per pass in each direction, far
// larger than L2) is loaded / stored non-temporally, so the gathers of L keep
// L2 to themselves (as the parity kernels' E stream; +2-3 %,
// profiles/r1u_nt/ab_phys_nt.txt).
__device__ __forceinline__ float ld_e32(const float *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_e32(float *p, float v) { __builtin_nontemporal_store(v, p); }


constexpr int kRowsPerWave = 4;
constexpr int kColsPerWave = 8;
constexpr int kVnBatch = 4;  // columns per batch of phys_vn_tile's batched loads (2 / 8: same or slower)

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Work item i = (tile, part).  Blocks b and b+8 run on the same XCD; the grid
// is a multiple of 8 and block b takes items b, b+G, b+2G, ... so every item
// of a block -- and every part of one tile -- has the same i%8 = tile%8: a
// tile's L rows stay in one XCD's L2.  A grid of a few thousand blocks makes
// a launch over finished tiles cost a few microseconds, not one block per item.
__device__ __forceinline__ void xcd_item(int i, int per_tile, int &tile, int &part) {
    const int slot = i >> 3;
    tile = (slot / per_tile) * 8 + (i & 7);
    part = slot % per_tile;
}

// ------------------------------------------------------- tile decoder
__global__ void phys_tile_init_kernel(DevGraph g, DevState st, PhysTile pt, int convert) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)st.ntiles * g.n * kTile;
    if (convert && i < total) pt.L[i] = pt.Lam[i] = -(float)st.ch[i];  // Lambda = log P0/P1 = -channel LLR
    if (i < (size_t)st.ntiles * kTile) {
        const int f = (int)i;
        const bool valid = f < st.count;
        st.done[f] = valid ? 0 : 2;  // 2: no frame (never counted)
        st.conv[f] = -1;
        st.status[f] = 1;
        st.iters[f] = 0;
        pt.bad[f] = 0;
        pt.bad[pt.cap + f] = 0;
        if ((f & 63) == 0) st.tile_active[f >> 6] = valid ? 1 : 0;
    }
}

// One row's update from its gathered posteriors Lc and messages Eo (E_old;
// unused on iteration 0, for a stopped frame or in the syndrome-only sweep):
// phi(|M|) and the signs in registers, E_new = sign * phi(S - phi(|M_i|)).
// Returns the row parity of the hard decisions (L < 0).
template <int kDeg>
__device__ __forceinline__ uint32_t phys_row(float *__restrict__ Et, int beg, int deg, const float (&Lc)[kDeg],
                                             const float (&Eo)[kDeg], bool first, bool live, bool syn_only) {
    uint32_t hp = 0u, sg = 0u;
    float ph[kDeg];
    float S = 0.0f;
#pragma unroll
    for (int i = 0; i < kDeg; ++i) {
        if (i < deg) {
            hp ^= Lc[i] < 0.0f ? 1u : 0u;
            if (!syn_only) {
                const float M = (first || !live) ? Lc[i] : Lc[i] - Eo[i];
                ph[i] = phi(fabsf(M));
                S += ph[i];
                sg |= (M < 0.0f ? 1u : 0u) << i;
            }
        }
    }
    if (!syn_only && live) {
        const uint32_t neg = __popc(sg) & 1u;
#pragma unroll
        for (int i = 0; i < kDeg; ++i) {
            if (i < deg) {
                const float mag = phi(fmaxf(S - ph[i], 0.0f));
                st_e32(&Et[(beg + i) * kTile], ((neg ^ (sg >> i)) & 1u) ? -mag : mag);
            }
        }
    }
    return hp;
}

// A wavefront takes kRowsPerWave rows of one tile, one after the other: rows
// of degree <= kDeg with their gathers and E_old loads issued together
// (phys_row), longer rows in two sweeps with M recomputed (same values).
// (Batching the loads of 2 or 4 rows before any row's math measured 1.5-3 %
// slower once phi was cheap: the extra registers cost occupancy,
// profiles/r6_ab/r6e_c5.)
template <int kDeg>
__global__ __launch_bounds__(256) void phys_cn_tile_kernel(DevGraph g, DevState st, PhysTile pt, int it,
                                                           int syn_only, int per_tile, int items,
                                                           const int *__restrict__ row_ptr,
                                                           const int *__restrict__ col_idx) {
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
    int tile, part;
    xcd_item(item, per_tile, tile, part);
    if (tile >= st.ntiles || !st.tile_active[tile]) continue;
    const int f = tile * kTile + lane;
    const bool live = st.done[f] == 0;
    const float *Lt = pt.L + (size_t)tile * g.n * kTile + lane;
    float *Et = pt.E + (size_t)tile * g.nnz * kTile + lane;
    const bool first = it == 0;
    const bool readE = !first && !syn_only && live;
    uint32_t bad = 0u;
    const int r0 = (part * 4 + wave) * kRowsPerWave;
    for (int rr = 0; rr < kRowsPerWave; ++rr) {
        const int r = r0 + rr;
        if (r >= g.m) break;
        const int beg = row_ptr[r], deg = row_ptr[r + 1] - beg;
        if (deg <= kDeg) {
            float Lc[kDeg], Eo[kDeg];
            // lane-masked loads: a tile with few running frames moves only
            // their sectors, not 256 B per wavefront access
#pragma unroll
            for (int i = 0; i < kDeg; ++i) {
                Lc[i] = 0.0f;
                Eo[i] = 0.0f;
                if (i < deg) {
                    if (live) Lc[i] = Lt[col_idx[beg + i] * kTile];
                    if (readE) Eo[i] = ld_e32(&Et[(beg + i) * kTile]);
                }
            }
            bad |= phys_row<kDeg>(Et, beg, deg, Lc, Eo, first, live, syn_only != 0);
        } else {
            const int end = beg + deg;
            uint32_t hp = 0u;
            float S = 0.0f;
            uint32_t neg = 0u;
            for (int e = beg; e < end; ++e) {
                const float Lc = live ? Lt[col_idx[e] * kTile] : 0.0f;
                hp ^= Lc < 0.0f ? 1u : 0u;
                if (!syn_only) {
                    const float M = (first || !live) ? Lc : Lc - Et[e * kTile];
                    S += phi(fabsf(M));
                    neg ^= (M < 0.0f) ? 1u : 0u;
                }
            }
            if (!syn_only && live) {
                for (int e = beg; e < end; ++e) {
                    const float Lc = Lt[col_idx[e] * kTile];
                    const float M = first ? Lc : Lc - ld_e32(&Et[e * kTile]);
                    const float mag = phi(fmaxf(S - phi(fabsf(M)), 0.0f));
                    st_e32(&Et[e * kTile], ((neg ^ ((M < 0.0f) ? 1u : 0u)) != 0u) ? -mag : mag);
                }
            }
            bad |= hp;
        }
    }
    // syndrome of the posterior of iteration it-1 (none before iteration 0)
    if (it >= 1 && live && bad) pt.bad[(it & 1) * pt.cap + f] = 1;
    }
}

// A wavefront takes kColsPerWave columns of one tile: L = Lambda + E_0 + E_1
// + ... in CSC order.  With every column of degree <= kCD (template; 0 = the
// plain loop for any degree), all the wavefront's message loads -- up to
// 8 x kCD -- are issued before the first sum (the per-column loop waited one
// memory latency per message: each add needs its load).
template <int kCD>
__global__ __launch_bounds__(256) void phys_vn_tile_kernel(DevGraph g, DevState st, PhysTile pt, int it,
                                                           int per_tile, int items, const int *__restrict__ csc_ptr,
                                                           const int *__restrict__ csc_edge, int *active_count,
                                                           int max_iter) {
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
    int tile, part;
    xcd_item(item, per_tile, tile, part);
    if (tile >= st.ntiles || !st.tile_active[tile]) continue;
    const int f = tile * kTile + lane;
    // done[f] may flip to 1 under us (the wave below): either value gives upd = 0
    const bool live = st.done[f] == 0;
    const bool conv_now = live && it >= 1 && pt.bad[(it & 1) * pt.cap + f] == 0;
    const bool upd = live && !conv_now;
    const float *Et = pt.E + (size_t)tile * g.nnz * kTile + lane;
    float *Lt = pt.L + (size_t)tile * g.n * kTile + lane;
    const float *Lamt = pt.Lam + (size_t)tile * g.n * kTile + lane;
    if (__ballot(upd) != 0ull) {
        const int j0 = (part * 4 + wave) * kColsPerWave;
        const int j1 = min(g.n, j0 + kColsPerWave);
        uint32_t hb = 0u;  // this lane's hard decisions of the 8 columns (early syndrome)
        if constexpr (kCD > 0) {
            // batches of CB columns (CB x kCD loads in flight; more batch
            // columns spill the uniform edge indices)
            constexpr int CB = kVnBatch;
#pragma unroll
            for (int b = 0; b < kColsPerWave / CB; ++b) {
                float Ev[CB][kCD], La[CB];
                int p0[CB], cd[CB];
#pragma unroll
                for (int q = 0; q < CB; ++q) {
                    const int j = j0 + b * CB + q;
                    p0[q] = j < j1 ? csc_ptr[j] : 0;
                    cd[q] = j < j1 ? csc_ptr[j + 1] - p0[q] : 0;
                }
                // lane-masked: converged / finished frames move no data
#pragma unroll
                for (int q = 0; q < CB; ++q) {
                    La[q] = 0.0f;
                    if (upd && cd[q] > 0) La[q] = Lamt[(j0 + b * CB + q) * kTile];
#pragma unroll
                    for (int i = 0; i < kCD; ++i) {
                        Ev[q][i] = 0.0f;
                        if (upd && i < cd[q]) Ev[q][i] = ld_e32(&Et[csc_edge[p0[q] + i] * kTile]);
                    }
                }
#pragma unroll
                for (int q = 0; q < CB; ++q) {
                    float sum = La[q];
#pragma unroll
                    for (int i = 0; i < kCD; ++i)
                        if (i < cd[q]) sum += Ev[q][i];
                    if (upd && j0 + b * CB + q < j1) Lt[(j0 + b * CB + q) * kTile] = sum;
                    hb |= (sum < 0.0f ? 1u : 0u) << (b * CB + q);
                }
            }
        } else {
            for (int j = j0; j < j1; ++j) {
                if (upd) {
                    float sum = Lamt[j * kTile];
                    for (int p = csc_ptr[j]; p < csc_ptr[j + 1]; ++p) sum += ld_e32(&Et[csc_edge[p] * kTile]);
                    Lt[j * kTile] = sum;
                    hb |= (sum < 0.0f ? 1u : 0u) << (j - j0);
                }
            }
        }
        if (j0 < g.n && upd) pt.zb[((size_t)tile * ((g.n + 7) >> 3) + (j0 >> 3)) * kTile + lane] = (uint8_t)hb;
    }
    if (part == 0 && wave == 0) {
        if (conv_now) {  // syndrome of iteration it-1 was zero
            st.done[f] = 1;
            st.conv[f] = it - 1;
            st.status[f] = 0;
            st.iters[f] = it;
        }
        pt.bad[((it + 1) & 1) * pt.cap + f] = 0;  // for the next CN sweep
        const unsigned long long any = __ballot(upd);
        if (lane == 0) {
            st.tile_active[tile] = any != 0ull ? 1 : 0;
            if (any) {
                atomicAdd(&active_count[it], 1);  // host polls: 0 -> every frame has stopped
                atomicAdd(&active_count[max_iter + it], (int)__popcll(any));  // running frames (compaction)
            }
        }
    }
    }
}

// Early syndrome: the row parities of the hard decisions VN(it) just wrote
// (pt.zb: one byte per 8 columns, kColsPerWave == 8), one wavefront per
// (tile, 4 rows) like phys_cn_tile, into bad[(it+1)&1] -- the flag CN(it+1)
// would set from the same posterior.  Then phys_tile_exit stops the frames
// whose flag stayed 0: converged at iteration it (the exit VN(it+1) would have
// taken, one CN sweep earlier).  Only the running frames' bytes are current.
static_assert(kColsPerWave == 8, "one hard-decision byte per VN wavefront");
__global__ __launch_bounds__(256) void phys_tile_syn_kernel(DevGraph g, DevState st, PhysTile pt, int it,
                                                            int per_tile, int items, const int *__restrict__ row_ptr,
                                                            const int *__restrict__ col_idx) {
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    const size_t nb = (size_t)(g.n + 7) >> 3;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        int tile, part;
        xcd_item(item, per_tile, tile, part);
        if (tile >= st.ntiles || !st.tile_active[tile]) continue;
        const int f = tile * kTile + lane;
        const bool live = st.done[f] == 0;
        if (__ballot(live) == 0ull) continue;
        const uint8_t *zt = pt.zb + (size_t)tile * nb * kTile + lane;
        uint32_t bad = 0u;
        const int r0 = (part * 4 + wave) * kRowsPerWave;
        for (int rr = 0; rr < kRowsPerWave; ++rr) {
            const int r = r0 + rr;
            if (r >= g.m) break;
            uint32_t hp = 0u;
            for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                const int c = col_idx[e];
                hp ^= ((uint32_t)zt[(size_t)(c >> 3) * kTile] >> (c & 7)) & 1u;
            }
            bad |= hp;
        }
        if (live && bad) pt.bad[((it + 1) & 1) * pt.cap + f] = 1;
    }
}
__global__ __launch_bounds__(64) void phys_tile_exit_kernel(DevState st, PhysTile pt, int it, int *active_count,
                                                            int max_iter) {
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int f = tile * kTile + lane;
    const bool live = st.tile_active[tile] && st.done[f] == 0;
    const bool conv_now = live && pt.bad[((it + 1) & 1) * pt.cap + f] == 0;
    if (conv_now) {  // the syndrome of iteration it is zero
        st.done[f] = 1;
        st.conv[f] = it;
        st.status[f] = 0;
        st.iters[f] = it + 1;
    }
    const unsigned long long still = __ballot(live && !conv_now);
    if (lane == 0) {
        if (st.tile_active[tile]) st.tile_active[tile] = still != 0ull ? 1 : 0;
        if (still) {
            atomicAdd(&active_count[it], 1);
            atomicAdd(&active_count[max_iter + it], (int)__popcll(still));
        }
    }
}

// after the syndrome-only sweep of "iteration" max_iter
__global__ void phys_tile_final_kernel(DevState st, PhysTile pt, int max_iter) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= st.ntiles * kTile || st.done[f]) return;
    const bool ok = pt.bad[(max_iter & 1) * pt.cap + f] == 0;
    st.done[f] = 1;
    st.conv[f] = ok ? max_iter - 1 : -1;
    st.status[f] = ok ? 0 : 1;
    st.iters[f] = max_iter;
}

// L32 tiles -> row-major z = (L < 0 ? 0 : 1) (bit estimate ^ 1) and post
__global__ void phys_tile_out_kernel(DevGraph g, DevState st, PhysTile pt, uint8_t *z, float *post) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)st.count * g.n) return;
    const int f = (int)(i / g.n);
    const int j = (int)(i % g.n);
    const float L = pt.L[((size_t)(f >> 6) * g.n + j) * kTile + (f & 63)];
    if (z) z[i] = L < 0.0f ? 0 : 1;
    if (post) post[i] = L;
}

// main.py counters; block = one wavefront x (tile, 1024 info columns)
__global__ __launch_bounds__(64) void phys_tile_count_kernel(DevGraph g, DevState st, PhysTile pt,
                                                             unsigned long long *ctr) {
    const int kw = (g.k + 31) >> 5;
    const int per_tile = (g.k + 1023) >> 10 > 0 ? (g.k + 1023) >> 10 : 1;
    const int tile = blockIdx.x / per_tile, part = blockIdx.x % per_tile;
    const int lane = threadIdx.x;
    const int f = tile * kTile + lane;
    const bool valid = st.done[f] == 1;  // finished and not counted yet (phys_tile_init, phys_compact)
    const bool failed = valid && st.status[f] != 0;
    unsigned long long err = 0;
    if (__ballot(failed) != 0ull) {  // BER counts failed frames only (main.py:130-138)
        const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
        const float *Lt = pt.L + (size_t)tile * g.n * kTile + lane;
        const int j1 = min(g.k, (part + 1) * 1024);
        for (int j = part * 1024; j < j1; ++j) {
            const uint32_t u = (Ut[(j >> 5) * kTile] >> (j & 31)) & 1u;
            err += (u != (Lt[j * kTile] < 0.0f ? 1u : 0u)) ? 1 : 0;
        }
        if (!failed) err = 0;
    }
    const unsigned long long e = wave_sum(err);
    if (lane == 0 && e) atomicAdd(&ctr[2], e);
    if (part != 0) return;
    const int cv = valid ? st.conv[f] : -1;
    unsigned long long v[7] = {valid ? 1ull : 0ull, failed ? 1ull : 0ull, 0, cv >= 0 ? (unsigned long long)cv : 0,
                               cv >= 0 ? 1ull : 0ull, 0, valid ? (unsigned long long)st.iters[f] : 0};
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        if (i == 2 || i == 5) continue;
        const unsigned long long s = wave_sum(v[i]);
        if (lane == 0 && s) atomicAdd(&ctr[i], s);
    }
}

// Compaction (Monte-Carlo runs): after the finished frames were counted,
// mark them counted; then move each running frame of the plan (spa_kernels
// compact plan: sources = running slots in tiles >= nt, destinations =
// finished slots below) -- its lanes of E32, L32, Lambda and the u bits --
// and reset the destination's per-frame state.  Sources and destinations are
// disjoint, so the moves need no ordering.
__global__ void phys_mark_counted_kernel(DevState st) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < st.ntiles * kTile && st.done[f] == 1) st.done[f] = 2;
}
__global__ void phys_compact_move_kernel(DevGraph g, DevState st, PhysTile pt, int cap, const int *pairs) {
    const int P = pairs[0];
    const int kw = (g.k + 31) >> 5;
    const int64_t items = (int64_t)g.nnz + 2 * (int64_t)g.n + kw;
    const int64_t total = (int64_t)P * items;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i % P);  // pair-fastest: neighbouring lanes of one item
        int64_t it = i / P;
        const int src = pairs[1 + p], dst = pairs[1 + cap + p];
        const size_t sT = src >> 6, sl = src & 63, dT = dst >> 6, dl = dst & 63;
        if (it < g.nnz) {
            pt.E[(dT * g.nnz + it) * kTile + dl] = pt.E[(sT * g.nnz + it) * kTile + sl];
            continue;
        }
        it -= g.nnz;
        if (it < g.n) {
            pt.L[(dT * g.n + it) * kTile + dl] = pt.L[(sT * g.n + it) * kTile + sl];
            continue;
        }
        it -= g.n;
        if (it < g.n) {
            pt.Lam[(dT * g.n + it) * kTile + dl] = pt.Lam[(sT * g.n + it) * kTile + sl];
            continue;
        }
        it -= g.n;
        st.ubits[(dT * kw + it) * kTile + dl] = st.ubits[(sT * kw + it) * kTile + sl];
    }
}
__global__ void phys_compact_flags_kernel(DevState st, PhysTile pt, int cap, const int *pairs) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= pairs[0]) return;
    const int src = pairs[1 + p], dst = pairs[1 + cap + p];
    st.done[dst] = 0;
    st.conv[dst] = -1;
    st.status[dst] = 1;
    st.iters[dst] = 0;
    pt.bad[dst] = 0;
    pt.bad[pt.cap + dst] = 0;
    st.tile_active[dst >> 6] = 1;
    st.done[src] = 2;  // moved: nothing to count here
}

inline unsigned grid_for(size_t total, int block) { return (unsigned)((total + block - 1) / block); }
inline unsigned xcd_items(int ntiles, int per_tile) { return (unsigned)(((ntiles + 7) / 8) * 8 * per_tile); }
// 256 CUs x 16 blocks of 4 waves (a multiple of 8, see xcd_item)
inline unsigned stride_grid(int items) { return (unsigned)std::min(items, 4096); }

}  // namespace

hipError_t launch_phys_tile_init(const DevGraph &g, const DevState &st, const PhysTile &pt, bool convert,
                                 hipStream_t s) {
    const size_t total = convert ? std::max((size_t)st.ntiles * g.n * kTile, (size_t)st.ntiles * kTile)
                                 : (size_t)st.ntiles * kTile;
    phys_tile_init_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, pt, convert ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_phys_tile_cn(const DevGraph &g, const DevState &st, const PhysTile &pt, int it, bool syn_only,
                               hipStream_t s) {
    const int per_tile = (g.m + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave);
    const int items = (int)xcd_items(st.ntiles, per_tile);
    const unsigned grid = stride_grid(items);
    const int so = syn_only ? 1 : 0;
    if (g.max_row_deg <= 8)
        phys_cn_tile_kernel<8><<<grid, 256, 0, s>>>(g, st, pt, it, so, per_tile, items, g.row_ptr, g.col_idx);
    else if (g.max_row_deg <= 16)
        phys_cn_tile_kernel<16><<<grid, 256, 0, s>>>(g, st, pt, it, so, per_tile, items, g.row_ptr, g.col_idx);
    else
        phys_cn_tile_kernel<32><<<grid, 256, 0, s>>>(g, st, pt, it, so, per_tile, items, g.row_ptr, g.col_idx);
    return hipGetLastError();
}

hipError_t launch_phys_tile_vn(const DevGraph &g, const DevState &st, const PhysTile &pt, int it, int *active_count,
                               int max_iter, hipStream_t s) {
    const int per_tile = (g.n + 4 * kColsPerWave - 1) / (4 * kColsPerWave);
    const int items = (int)xcd_items(st.ntiles, per_tile);
    if (g.max_col_deg <= 8)
        phys_vn_tile_kernel<8><<<stride_grid(items), 256, 0, s>>>(g, st, pt, it, per_tile, items, g.csc_ptr,
                                                                  g.csc_edge, active_count, max_iter);
    else
        phys_vn_tile_kernel<0><<<stride_grid(items), 256, 0, s>>>(g, st, pt, it, per_tile, items, g.csc_ptr,
                                                                  g.csc_edge, active_count, max_iter);
    return hipGetLastError();
}

hipError_t launch_phys_tile_final(const DevGraph &, const DevState &st, const PhysTile &pt, int max_iter,
                                  hipStream_t s) {
    phys_tile_final_kernel<<<grid_for((size_t)st.ntiles * kTile, 256), 256, 0, s>>>(st, pt, max_iter);
    return hipGetLastError();
}

hipError_t launch_phys_tile_out(const DevGraph &g, const DevState &st, const PhysTile &pt, uint8_t *z, float *post,
                                hipStream_t s) {
    const size_t total = (size_t)st.count * g.n;
    if (total && (z || post)) phys_tile_out_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, pt, z, post);
    return hipGetLastError();
}

hipError_t launch_phys_tile_early_exit(const DevGraph &g, const DevState &st, const PhysTile &pt, int it,
                                       int *active_count, int max_iter, hipStream_t s) {
    const int per_tile = (g.m + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave);
    const int items = (int)xcd_items(st.ntiles, per_tile);
    phys_tile_syn_kernel<<<stride_grid(items), 256, 0, s>>>(g, st, pt, it, per_tile, items, g.row_ptr, g.col_idx);
    if (hipError_t e = hipMemsetAsync(active_count + it, 0, sizeof(int), s)) return e;
    if (hipError_t e = hipMemsetAsync(active_count + max_iter + it, 0, sizeof(int), s)) return e;
    phys_tile_exit_kernel<<<st.ntiles, kTile, 0, s>>>(st, pt, it, active_count, max_iter);
    return hipGetLastError();
}

hipError_t launch_phys_compact(const DevGraph &g, const DevState &st, const PhysTile &pt, int nt, int cap, int *pairs,
                               hipStream_t s) {
    phys_mark_counted_kernel<<<grid_for((size_t)st.ntiles * kTile, 256), 256, 0, s>>>(st);
    if (hipError_t e = launch_compact_plan(st, nt, cap, pairs, s)) return e;
    phys_compact_move_kernel<<<2048, 256, 0, s>>>(g, st, pt, cap, pairs);
    phys_compact_flags_kernel<<<grid_for((size_t)cap, 256), 256, 0, s>>>(st, pt, cap, pairs);
    return hipGetLastError();
}

hipError_t launch_phys_tile_count(const DevGraph &g, const DevState &st, const PhysTile &pt,
                                  unsigned long long *ctr, hipStream_t s) {
    const int per_tile = std::max(1, (g.k + 1023) >> 10);
    phys_tile_count_kernel<<<st.ntiles * per_tile, 64, 0, s>>>(g, st, pt, ctr);
    return hipGetLastError();
}

}  // namespace ldpc
