// spa_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the SPA decoder.
//
// One decode iteration of python_ldpc_app/spa_decoder.py:104-276 is two
// launches over a chunk of frame tiles (layout: spa_device.h):
//
//   cn_kernel  one wavefront per (tile, check row).  Lane = frame.  Walks the
//              row's edges in ascending column order (the reference's
//              check_to_var order) and reproduces spa_decoder.py:112-168 and
//              the M update :260-268 fused in front of it:
//                M = L[col] - E_old      (iteration 0: M = ch[col], :85-90)
//                t = tanh(M/2) with the +-17.5 clip            (:138-146)
//                P = t0*t1*...  strictly left to right          (np.prod, :152)
//                q = P/t (|t|>1e-10) else prod of the others    (:159-164)
//                E = 2*atanh(clip(q, +-CL))                     (:167-168)
//              Pass 1 only forms P; pass 2 recomputes t from the same E_old
//              and L bits (24 B of HBM traffic per edge, not 32 B for parking
//              t).  A wavefront holding some |t| <= 1e-10 instead parks t in a
//              scratch array T, because the rare "product of the others"
//              branch re-reads every t while E is overwritten in place.
//   vn_kernel  one workgroup (16 wavefronts) per tile; wavefront w takes
//              columns w, w+16, ...:
//                L = ch + ((0+E[r0])+E[r1])+...  rows ascending (:173-185)
//                z = L<0                                         (:188)
//              and FUSES the early-termination syndrome (:191-204): every
//              lane XORs its (z^1) into the m-bit row-parity vector of its
//              frame held in LDS ([m/32][64] words, ds_xor_b32), then one
//              wavefront ORs the words: zero -> converged at this iteration
//              (:231-241), else NOT_OK at the last iteration (:244-253).
//              The normalized-LLR count (:210-228) is fused here as well.
//
// Numerics: fp64 throughout; this file is compiled with -ffp-contract=off and
// without fast-math, so every +,-,*,/ is one correctly rounded IEEE op in the
// reference's order.  tanh is numpy's own float64 algorithm (bit-identical
// to the reference's np.tanh); atanh is correctly rounded on > 99% of inputs
// (spa_math.h).  Their coefficient tables are staged in LDS per block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "frame_source.h"
#include "spa_device.h"
#include "cn_common.h"
#include "spa_math.h"

namespace ldpc {
namespace {

constexpr int kCnRowsPerBlock = 4;           // 4 wavefronts = 4 rows of one tile
constexpr int kVnWaves = 16;                 // wavefronts per VN workgroup
constexpr int kPv = 4;                       // VN column-sum loads in flight

// --------------------------------------------------------------- CN pass
constexpr int kCnWaves = 7;  // min wavefronts per SIMD for cn_kernel (register budget)
constexpr int kPf = 4;       // edges in flight per wavefront (software pipeline depth; 6 and 8 measured no faster, profiles/r3_ab/ab_pf)

// The message array E (streamed once per pass, far larger than L2) is loaded
// and stored non-temporally by the CN/VN kernels, so it does not evict the
// tiles' posteriors (the L[col] gather) from L2 (profiles/r1u_nt).
__device__ __forceinline__ double ld_e(const double *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_e(double *p, double v) { __builtin_nontemporal_store(v, p); }

// Register ring of the next kPf edges' (L[col], E_old) loads.  take(k, e)
// returns M for edge e (ring slot k) and issues the loads for edge e + kPf.
// kStream (streaming Monte-Carlo): a lane whose frame was just loaded
// ("fresh", L = ch) takes M = L - 0 -- its iteration 0 -- while the other
// lanes of the wavefront take M = L - E_old.
template <bool kFirst, bool kStream>
struct EdgeStream {
    const int *__restrict__ col;
    const double *Lt, *Et;
    int end, es;  // es: E stride between edges (DevGraph::ef)
    bool fresh;
    double lv[kPf], eo[kPf];
    __device__ __forceinline__ EdgeStream(const int *__restrict__ col_, const double *L_, const double *E_, int beg,
                                          int end_, bool fresh_, int es_)
        : col(col_), Lt(L_), Et(E_), end(end_), es(es_), fresh(fresh_) {
#pragma unroll
        for (int k = 0; k < kPf; ++k) fetch(k, beg + k);
    }
    __device__ __forceinline__ void fetch(int k, int e) {
        // unconditional (index clamped into the row): no phi, so the compiler
        // keeps the ring in place and waits only for the slot it consumes
        const int i = e < end ? e : end - 1;
        lv[k] = Lt[col[i] * kTile];  // col[] is read-only + noalias -> scalar load
        eo[k] = kFirst ? 0.0 : ld_e(&Et[(size_t)i * es]);
    }
    __device__ __forceinline__ double take(int k, int e) {
        const double M = kFirst ? lv[k] : lv[k] - ((kStream && fresh) ? 0.0 : eo[k]);
        fetch(k, e + kPf);
        return M;
    }
};
template <bool kFirst, bool kStream>
__global__ __launch_bounds__(256, kCnWaves) void cn_kernel(DevGraph g, DevState st, int blocks_per_tile,
                                                                int it_parity, const int *__restrict__ col_idx,
                                                                const int *__restrict__ row_ptr, AtanhCoef ac) {
    __shared__ MathLds mlds;
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    // XCD-aware mapping: blocks b and b+8 share an XCD (round-robin dispatch),
    // so give every block of one tile the same b%8: the tile's L/ch rows
    // (gathered by every check row) then stay in that XCD's L2.
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int tile = (slot / blocks_per_tile) * 8 + (b & 7);
    const int row = (slot % blocks_per_tile) * kCnRowsPerBlock + wave;
    // block-uniform: a block of a finished (or padding) tile leaves before
    // staging the math tables
    if (tile >= st.ntiles || !st.tile_active[tile]) return;
    fill_math_lds(mlds);
    __syncthreads();
    const LdsTanh ttab{mlds.tanh};
    const LdsAtanh ltab{mlds.atanh};
    if (row >= g.m) return;
    const int beg = row_ptr[row], end = row_ptr[row + 1];
    if (beg == end) return;  // spa_decoder.py:115-122

    const int f = tile * kTile + lane;
    const bool live = st.done[f] == 0;
    const bool fresh = kStream && st.fresh[f] != 0;
    double *Et = st.E + e_base(g, tile, lane);
    const double *Lt = (kFirst ? st.ch : st.L) + (size_t)tile * g.n * kTile + lane;

    // Both passes stream (L[col], E_old) through a register ring of kPf
    // edges, so kPf edges' loads are in flight per wavefront.
    // pass 1: P = t0*t1*... left to right; nothing is stored
    double P = 1.0;
    bool tiny = false;
    {
        EdgeStream<kFirst, kStream> es(col_idx, Lt, Et, beg, end, fresh, g.ef);
        for (int e = beg; e < end; e += kPf) {
#pragma unroll
            for (int k = 0; k < kPf; ++k) {
                const double M = es.take(k, e + k);
                if (e + k < end) {  // wave-uniform
                    const double t = cn_tanh(M, ttab);
                    P = (e + k == beg) ? t : P * t;
                    tiny |= live && !(fabs(t) > kTiny);  // a frame-less lane never votes
                }
            }
        }
    }
    if (__ballot(tiny) == 0ull) {
        // pass 2: recompute t from the same E_old / L bits (identical result),
        // E_new = 2 atanh(clip(P/t)) written over E_old.  24 B of HBM per edge
        // instead of parking t (32 B).
        EdgeStream<kFirst, kStream> es(col_idx, Lt, Et, beg, end, fresh, g.ef);
        const bool nr = div_nr_ok(live ? P : 1.0);  // wave-uniform (cn_common.h); frame-less lanes do not vote
        const double lim = live ? kAtanhIdent : INFINITY;
        for (int e = beg; e < end; e += kPf) {
#pragma unroll
            for (int k = 0; k < kPf; ++k) {
                const double M = es.take(k, e + k);
                if (e + k < end) {  // wave-uniform
                    const double t = cn_tanh(M, ttab);
                    const double q = nr ? div_nr(P, t) : P / t;
                    // 2q where exact for the whole wavefront (spa_math.h kAtanhIdent)
                    const double En = __ballot(!(fabs(q) < lim)) == 0ull
                                          ? 2.0 * q
                                          : 2.0 * atanh_f(clip_cl(q), ltab, ac);
                    if (live) st_e(&Et[(size_t)(e + k) * g.ef], En);
                }
            }
        }
        return;
    }
    // Rare: some |t| <= 1e-10 in this wavefront.  Leave E untouched and hand
    // the row to cn_rare_kernel (next launch), which needs every t of the row
    // while overwriting E and so parks them in a scratch slot.
    if (lane == 0) {
        const int at = atomicAdd(&st.rare_count[it_parity], 1);
        st.rare_list[at] = tile * g.m + row;
    }
}

// ------------------------------------------------- CN pass, row in registers
// One workgroup of W = 8 wavefronts per (tile, check row), for rows of degree
// <= W*K = 192 (every row of wimax_576_0.5).  Wavefront w owns the contiguous
// edges [beg + w*C, beg + (w+1)*C), C = ceil(deg/W), and keeps their t in
// registers (K fp64 each, statically indexed):
//   phase 1  issue all its loads of L[col] and E_old at once (unconditional,
//            index clamped into the chunk), then t = tanh(M/2)   (8 B/edge read)
//   phase 2  P = t0*t1*...*t_{deg-1} strictly left to right: wavefront 0
//            multiplies its chunk, hands the running product to wavefront 1
//            through LDS, ... (W barriers; the reference's rounding order)
//   phase 3  E_new = 2 atanh(clip(P/t)) from the register t    (8 B/edge write)
// = the algorithmic 16 B/edge, and tanh is evaluated once per edge (cn_kernel
// re-reads E_old and recomputes t in its pass 2).  A row where some lane has
// |t| <= 1e-10 goes to cn_rare_kernel untouched, as in cn_kernel.
// Phase 1 issues its loads in S stages of K/S edges, so the workgroup fits in
// 80 registers and three run per CU (latency hiding: the product chain parks
// 7 of 8 wavefronts, phase 1 waits on HBM).  A/B on wimax_576_0.5
// (tools/ab_cnrow.sh, profiles/r1f_cnrow_s4): 10.5 ms vs 11.3 ms for all
// loads at once at 4 waves/SIMD and 14.2 ms for cn_kernel; 3 stages tie;
// W=4/K=48, W=16/K=12, 8-waves/SIMD shapes (spills) and persistent
// workgroups were slower.
constexpr int kRowW = 8, kRowK = 24;
// S: phase-1 load stages (K/S edges' loads in flight per stage); WPS: min
// wavefronts per SIMD (register cap 512/WPS).
// W, K: a second shape, 16 wavefronts x 40 edges (rows <= 640: wimax_2304_0.5,
// 416-632), serves the 2304 code's split path and its streaming tail.
template <bool kFirst, bool kStream, int S, int WPS, int W = kRowW, int K = kRowK>
__global__ __launch_bounds__(64 * W, WPS) void cn_row_kernel(DevGraph g, DevState st, int it_parity,
                                                             const int *__restrict__ col_idx,
                                                             const int *__restrict__ row_ptr, AtanhCoef ac) {
    __shared__ MathLds mlds;
    __shared__ double chain[kTile];  // running product handed from wavefront to wavefront
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    const int b = blockIdx.x;  // XCD-aware: every row of a tile on the tile's XCD
    const int slot = b >> 3;
    const int tile = (slot / g.m) * 8 + (b & 7);
    const int row = slot % g.m;
    if (tile >= st.ntiles || !st.tile_active[tile]) return;  // block-uniform, before the table staging
    fill_math_lds(mlds);
    __syncthreads();
    const LdsTanh ttab{mlds.tanh};
    const LdsAtanh ltab{mlds.atanh};
    const int beg = row_ptr[row], end = row_ptr[row + 1];
    const int deg = end - beg;
    if (deg == 0) return;  // spa_decoder.py:115-122
    const int f = tile * kTile + lane;
    const bool live = st.done[f] == 0;
    const bool fresh = kStream && st.fresh[f] != 0;
    double *Et = st.E + e_base(g, tile, lane);
    const double *Lt = (kFirst ? st.ch : st.L) + (size_t)tile * g.n * kTile + lane;
    const int C = (deg + W - 1) / W;
    const int c0 = beg + wave * C;
    const int cnt = max(0, min(end, c0 + C) - c0);  // wave-uniform, <= K (host checks deg <= W*K)

    double t[K];
    bool tiny = false;
    if (cnt > 0) {
#pragma unroll
        for (int h = 0; h < S; ++h) {
            constexpr int H = K / S;
            double eo[H];
#pragma unroll
            for (int i = h * H; i < (h + 1) * H; ++i) {
                const int e = c0 + min(i, cnt - 1);
                t[i] = Lt[col_idx[e] * kTile];
                eo[i - h * H] = kFirst ? 0.0 : ld_e(&Et[(size_t)e * g.ef]);
            }
#pragma unroll
            for (int i = h * H; i < (h + 1) * H; ++i) {
                if (i < cnt) {
                    const double M = kFirst ? t[i] : t[i] - ((kStream && fresh) ? 0.0 : eo[i - h * H]);
                    t[i] = cn_tanh(M, ttab);
                    tiny |= live && !(fabs(t[i]) > kTiny);
                }
            }
        }
    }
    if (__syncthreads_or(tiny)) {  // rare: the whole row to cn_rare_kernel
        if (threadIdx.x == 0) {
            const int at = atomicAdd(&st.rare_count[it_parity], 1);
            st.rare_list[at] = tile * g.m + row;
        }
        return;
    }
    for (int w = 0; w < W; ++w) {  // the product chain, in edge order
        if (wave == w && cnt > 0) {
            double P = w == 0 ? t[0] : chain[lane];
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < cnt && (w != 0 || i != 0)) P = P * t[i];
            chain[lane] = P;
        }
        __syncthreads();
    }
    const double P = chain[lane];
    // q = P/t (div_nr: the IEEE quotient without the scaling steps,
    // cn_common.h); E_new = 2 atanh(clip(q)), or 2q when every quotient of the
    // wavefront is below 2^-27 (exact: spa_math.h kAtanhIdent), edge by edge
    const double lim = live ? kAtanhIdent : INFINITY;  // frame-less lanes do not vote
    auto en = [&](double q) {
        return __ballot(!(fabs(q) < lim)) == 0ull ? 2.0 * q : 2.0 * atanh_f(clip_cl(q), ltab, ac);
    };
    if (div_nr_ok(live ? P : 1.0)) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if (i < cnt) {
                const double En = en(div_nr(P, t[i]));
                if (live) st_e(&Et[(size_t)(c0 + i) * g.ef], En);
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (i < cnt) {
            const double En = en(P / t[i]);
            if (live) st_e(&Et[(size_t)(c0 + i) * g.ef], En);
        }
    }
}

// Rows recorded by cn_kernel: same update, with t parked in this wavefront's
// own scratch slot (slot = global wavefront id; grid-stride over the list).
template <bool kFirst, bool kStream>
__global__ __launch_bounds__(256) void cn_rare_kernel(DevGraph g, DevState st, int it_parity, AtanhCoef ac) {
    __shared__ MathLds mlds;
    const int count = st.rare_count[it_parity];
    if (blockIdx.x == 0 && threadIdx.x == 0) st.rare_count[it_parity ^ 1] = 0;  // for the next CN
    if (count == 0) return;  // block-uniform
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.rare_count[2], count);  // ldpc_rare_rows_read
    fill_math_lds(mlds);
    __syncthreads();
    const LdsTanh ttab{mlds.tanh};
    const LdsAtanh ltab{mlds.atanh};
    const int lane = threadIdx.x & 63;
    const int gw = (int)blockIdx.x * 4 + uniform(threadIdx.x >> 6);
    const int nw = (int)gridDim.x * 4;
    double *Tt = st.T + (size_t)gw * g.max_row_deg * kTile + lane;
    for (int idx = gw; idx < count; idx += nw) {
        const uint32_t code = (uint32_t)st.rare_list[idx];
        const int tr = (int)(code & 0x0fffffffu);
        const uint32_t subs = code >> 28;  // 0: every frame of the tile; else the listed 16-frame sub-tiles
        const int tile = tr / g.m, row = tr % g.m;
        const int beg = g.row_ptr[row], end = g.row_ptr[row + 1];
        const int f = tile * kTile + lane;
        const bool mine = subs == 0u || ((subs >> (lane >> 4)) & 1u) != 0u;
        const bool live = mine && st.done[f] == 0;
        const bool fresh = kStream && st.fresh[f] != 0;
        double *Et = st.E + e_base(g, tile, lane);
        const double *Lt = (kFirst ? st.ch : st.L) + (size_t)tile * g.n * kTile + lane;
        double P = 1.0;
        for (int e = beg; e < end; ++e) {
            double M = Lt[g.col_idx[e] * kTile];
            if (!kFirst) M = M - (fresh ? 0.0 : Et[(size_t)e * g.ef]);
            const double t = cn_tanh(M, ttab);
            P = (e == beg) ? t : P * t;
            Tt[(e - beg) * kTile] = t;
        }
        for (int e = beg; e < end; ++e) {
            const double t = Tt[(e - beg) * kTile];
            double q;
            if (fabs(t) > kTiny) {
                q = P / t;
            } else {  // np.prod(np.delete(tanh_array, idx)) (spa_decoder.py:164)
                q = 1.0;
                bool first = true;
                for (int e2 = beg; e2 < end; ++e2) {
                    if (e2 == e) continue;
                    const double t2 = Tt[(e2 - beg) * kTile];
                    q = first ? t2 : q * t2;
                    first = false;
                }
            }
            const double En = 2.0 * atanh_f(clip_cl(q), ltab, ac);
            if (live) Et[(size_t)e * g.ef] = En;
        }
    }
}

// ------------------------------------------------------- VN + syndrome pass


// kStream (streaming Monte-Carlo): every lane is at its own iteration
// (iters[f] = iterations its frame has completed); `last` is max_iter.  A
// frame that finishes here adds its counters (count_kernel's definitions) to
// ctr and flags its lane for refill_kernel.
template <bool kFirst, bool kStream>
__global__ __launch_bounds__(1024) void vn_kernel(DevGraph g, DevState st, int it, int last, int nllr,
                                                  const int *__restrict__ csc_ptr,
                                                  const int *__restrict__ csc_edge,
                                                  const int *__restrict__ csc_row, unsigned long long *ctr) {
    extern __shared__ uint32_t par[];  // [mw][64] row parities of z^1, one column per frame
    __shared__ int cnt_lds[kTile];
    __shared__ int err_lds[kTile];
    const int tile = blockIdx.x;
    if (!st.tile_active[tile]) return;
    const int mw = (g.m + 31) >> 5;
    for (int i = threadIdx.x; i < mw * kTile; i += blockDim.x) par[i] = 0u;
    if (threadIdx.x < kTile) {
        cnt_lds[threadIdx.x] = 0;
        err_lds[threadIdx.x] = 0;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    const int f = tile * kTile + lane;
    const bool live = st.done[f] == 0;
    const int itl = kStream ? st.iters[f] : it;  // this lane's iteration
    const bool lastl = kStream ? (itl == last - 1) : (last != 0);
    // error bits are only needed by a frame that may fail at this iteration
    const bool want_err = kStream && __ballot(live && lastl) != 0ull;
    const int kw = (g.k + 31) >> 5;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
    int my_err = 0;
    const double *Et = st.E + e_base(g, tile, lane);
    double *Lt = st.L + (size_t)tile * g.n * kTile + lane;
    const double *Ct = st.ch + (size_t)tile * g.n * kTile + lane;

    int my_cnt = 0;
    for (int j = wave; j < g.n; j += nwaves) {
        const int p0 = csc_ptr[j], p1 = csc_ptr[j + 1];
        double s = 0.0;  // scipy csr_matvec: sum starts at y[i] = 0, rows ascending
        {
            // ring of kPv loads in flight (indices clamped into the column)
            double ring[kPv];
#pragma unroll
            for (int k = 0; k < kPv; ++k) ring[k] = ld_e(&Et[(size_t)csc_edge[min(p0 + k, p1 - 1)] * g.ef]);
            for (int p = p0; p < p1; p += kPv) {
#pragma unroll
                for (int k = 0; k < kPv; ++k) {
                    const double v = ring[k];
                    ring[k] = ld_e(&Et[(size_t)csc_edge[min(p + k + kPv, p1 - 1)] * g.ef]);
                    if (p + k < p1) s = s + v;
                }
            }
        }
        const double chj = Ct[j * kTile];
        const double Lj = chj + s;  // channel added after the sum (:173,185)
        if (nllr && j < g.k) {
            const double ap = kFirst ? chj : Lt[j * kTile];  // a-priori = previous L (:274)
            my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
        }
        if (want_err && j < g.k)
            my_err += (int)(((Ut[(j >> 5) * kTile] >> (j & 31)) & 1u) ^ (Lj < 0.0 ? 0u : 1u));  // u vs z^1
        if (live) Lt[j * kTile] = Lj;
        if (!(Lj < 0.0)) {  // z^1 == 1 -> flips the parity of every row of column j
            for (int p = p0; p < p1; ++p) {
                const int r = csc_row[p];
                atomicXor(&par[(r >> 5) * kTile + lane], 1u << (r & 31));
            }
        }
    }
    if (nllr) atomicAdd(&cnt_lds[lane], my_cnt);
    if (want_err) atomicAdd(&err_lds[lane], my_err);
    __syncthreads();
    if (wave != 0) return;

    uint32_t acc = 0u;
    for (int w = 0; w < mw; ++w) acc |= par[w * kTile + lane];
    bool still = false;
    if (kStream) {
        unsigned long long v[7] = {0, 0, 0, 0, 0, 0, 0};
        bool fin = false;
        if (live) {
            const bool ok = acc == 0u;
            fin = ok || lastl;
            if (fin) {
                v[0] = 1;
                v[1] = ok ? 0 : 1;
                v[2] = ok ? 0 : (unsigned long long)err_lds[lane];
                v[3] = ok ? (unsigned long long)itl : 0;
                v[4] = ok ? 1 : 0;
                v[5] = nllr ? (unsigned long long)cnt_lds[lane] : 0;
                v[6] = (unsigned long long)(itl + 1);
                st.done[f] = 1;
                st.refill[f] = 1;
            } else {
                st.iters[f] = itl + 1;
                still = true;
            }
            st.fresh[f] = 0;
        }
        if (__ballot(fin) != 0ull) {
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                const unsigned long long s = wave_sum(v[i]);
                if (lane == 0 && s) atomicAdd(&ctr[i], s);
            }
        }
    } else if (live) {
        if (nllr) {
            const int c = cnt_lds[lane];
            st.nllr_cnt[f] = c;
            if (st.nllr_hist) st.nllr_hist[(size_t)f * st.hist_stride + it] = g.k > 0 ? (double)c / g.k : 0.0;
        }
        if (acc == 0u) {  // syndrome zero: Result.OK at this iteration
            st.done[f] = 1;
            st.conv[f] = it;
            st.status[f] = 0;
            st.iters[f] = it + 1;
        } else if (last) {  // Result.DATA_TRANSFER_NOT_OK
            st.done[f] = 1;
            st.conv[f] = -1;
            st.status[f] = 1;
            st.iters[f] = it + 1;
        } else {
            still = true;
        }
    }
    const unsigned long long any = __ballot(still);
    if (lane == 0) {
        st.tile_active[tile] = any != 0ull ? 1 : 0;
        if (any && st.active_count) atomicAdd(&st.active_count[it], 1);  // host poll: 0 -> all stopped
    }
}

// ----------------------------------------- streaming tail: column-parallel VN
// vn_kernel runs one workgroup per tile, so with a handful of tiles left (the
// drain of the streaming schedule) an iteration costs ~11 ms of one CU's
// latency (profiles/r2au_tail).  The tail pair spreads a tile's columns over
// the chip instead: vn_cols_kernel, one wavefront per (tile, column) -- the
// column sum in rows-ascending CSC order (:173-185, scipy csr_matvec's order,
// loads kept kTv deep ahead of the sequential adds), L, the normalized-LLR
// count (:210-228) and the z^1 bit OR-ed into zb [tile][nw][64]; then
// tail_exit_kernel, one workgroup per tile: the syndrome (:191-204) as
// popcount(A_r & (z^1)_A) + (z^1)_{k+r} from the bit-packed rows, and exactly
// vn_kernel<.., kStream>'s per-frame exits and counters (main.py:130-138).
// zb and cnt are all-zero between iterations (tail_exit clears its tile).
constexpr int kTv = 16;
__global__ __launch_bounds__(256) void vn_cols_kernel(DevGraph g, DevState st, int nllr, uint32_t *zb, int *cnt,
                                                      int first) {
    const int tile = blockIdx.y;
    const int j = blockIdx.x * 4 + (int)(threadIdx.x >> 6);  // column (uniform per wavefront)
    if (j >= g.n || !st.tile_active[tile]) return;
    const int lane = threadIdx.x & 63;
    const int f = tile * kTile + lane;
    const bool live = st.done[f] == 0;
    const double *Et = st.E + e_base(g, tile, lane);
    const int p0 = g.csc_ptr[j], p1 = g.csc_ptr[j + 1];
    double s = 0.0;  // rows ascending, starting at 0.0
    double ring[kTv];
#pragma unroll
    for (int q = 0; q < kTv; ++q) ring[q] = Et[(size_t)g.csc_edge[min(p0 + q, p1 - 1)] * g.ef];
    for (int p = p0; p < p1; p += kTv) {
#pragma unroll
        for (int q = 0; q < kTv; ++q) {
            const double v = ring[q];
            ring[q] = Et[(size_t)g.csc_edge[min(p + q + kTv, p1 - 1)] * g.ef];
            if (p + q < p1) s = s + v;
        }
    }
    const size_t ci = ((size_t)tile * g.n + j) * kTile + lane;
    const double chj = st.ch[ci];
    const double Lj = chj + s;  // channel added after the sum
    if (nllr && j < g.k) {
        // previous posterior: ch on iteration 0 of a decode (L not yet written,
        // vn_kernel<true>), L = ch on a streaming frame's first pass
        const double ap = first ? chj : st.L[ci];
        if (fabs(Lj) <= 7.0 && ap * Lj < 0.0) atomicAdd(&cnt[f], 1);
    }
    if (live) st.L[ci] = Lj;
    if (!(Lj < 0.0)) {
        const int nw = (g.n + 31) >> 5;
        atomicOr(&zb[((size_t)tile * nw + (j >> 5)) * kTile + lane], 1u << (j & 31));
    }
}

constexpr int kTailWaves = 16;
constexpr int kTailKw = 64;  // (z^1)_A words held per lane: k <= 2048
// kDecode (ldpc_decode_f64 on few tiles, run_iterations): `it` is the pass,
// `last` whether it is the final one, and the exits are vn_kernel<.., false>'s
// (conv / status / iters, the normalized-LLR history, the host poll's count);
// otherwise `last` is max_iter and the exits are the streaming ones.
// gbad (decode only, may be null): the row parities were already OR-ed into
// gbad[frame] by syn_kernel (edge_kernels.hip); read and cleared here.
template <bool kDecode>
__global__ __launch_bounds__(64 * kTailWaves) void tail_exit_kernel(DevGraph g, DevState st, int it, int last,
                                                                     int nllr, uint32_t *zb, int *cnt,
                                                                     unsigned long long *ctr, int *gbad) {
    __shared__ int bad[kTile];
    const int tile = blockIdx.x;
    if (!st.tile_active[tile]) return;  // block-uniform
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int f = tile * kTile + lane;
    const int kw = (g.k + 31) >> 5, nw = (g.n + 31) >> 5;
    uint32_t *zt = zb + (size_t)tile * nw * kTile + lane;
    if (threadIdx.x < kTile) bad[threadIdx.x] = (kDecode && gbad) ? gbad[f] : 0;
    __syncthreads();
    uint32_t za[kTailKw];
    if (!(kDecode && gbad)) {
#pragma unroll
        for (int w = 0; w < kTailKw; ++w) {
            uint32_t v = w < kw ? zt[w * kTile] : 0u;
            if (w == kw - 1 && (g.k & 31)) v &= (1u << (g.k & 31)) - 1u;  // A columns only
            za[w] = v;
        }
        uint32_t acc = 0u;
        for (int r = wave; r < g.m; r += kTailWaves) {
            const uint32_t *ar = g.a_packed + (size_t)r * kw;
            const int q = g.k + r;  // identity column of row r
            uint32_t par = zt[(q >> 5) * kTile] >> (q & 31);
#pragma unroll
            for (int w = 0; w < kTailKw; ++w)
                if (w < kw) par += __builtin_popcount(ar[w] & za[w]);
            acc |= par & 1u;
        }
        if (acc) atomicOr(&bad[lane], 1);
    }
    __syncthreads();
    if (kDecode && wave == 0) {  // vn_kernel<.., false>'s exits
        const bool live = st.done[f] == 0;
        bool still = false;
        if (live) {
            if (nllr) {
                const int c = cnt[f];
                st.nllr_cnt[f] = c;
                if (st.nllr_hist) st.nllr_hist[(size_t)f * st.hist_stride + it] = g.k > 0 ? (double)c / g.k : 0.0;
            }
            if (bad[lane] == 0) {  // syndrome zero: Result.OK at this iteration
                st.done[f] = 1;
                st.conv[f] = it;
                st.status[f] = 0;
                st.iters[f] = it + 1;
            } else if (last) {  // Result.DATA_TRANSFER_NOT_OK
                st.done[f] = 1;
                st.conv[f] = -1;
                st.status[f] = 1;
                st.iters[f] = it + 1;
            } else {
                still = true;
            }
        }
        const unsigned long long any = __ballot(still);
        if (lane == 0) {
            st.tile_active[tile] = any != 0ull ? 1 : 0;
            if (any && st.active_count) atomicAdd(&st.active_count[it], 1);  // host poll: 0 -> all stopped
        }
        cnt[f] = 0;
        if (gbad) gbad[f] = 0;
    }
    if (!kDecode && wave == 0) {  // vn_kernel<false, true>'s exits and counters
        const bool live = st.done[f] == 0;
        const int itl = st.iters[f];
        const bool lastl = itl == last - 1;
        unsigned long long v[7] = {0, 0, 0, 0, 0, 0, 0};
        bool fin = false, still = false;
        if (live) {
            const bool ok = bad[lane] == 0;
            fin = ok || lastl;
            if (fin) {
                unsigned long long err = 0;
                if (!ok) {  // u vs z^1 of the info columns (main.py:130-138)
                    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;
#pragma unroll
                    for (int w = 0; w < kTailKw; ++w)
                        if (w < kw) err += __builtin_popcount(Ut[w * kTile] ^ za[w]);
                }
                v[0] = 1;
                v[1] = ok ? 0 : 1;
                v[2] = ok ? 0 : err;
                v[3] = ok ? (unsigned long long)itl : 0;
                v[4] = ok ? 1 : 0;
                v[5] = nllr ? (unsigned long long)cnt[f] : 0;
                v[6] = (unsigned long long)(itl + 1);
                st.done[f] = 1;
                st.refill[f] = 1;
            } else {
                st.iters[f] = itl + 1;
                still = true;
            }
            st.fresh[f] = 0;
        }
        if (__ballot(fin) != 0ull) {
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                const unsigned long long sm = wave_sum(v[i]);
                if (lane == 0 && sm) atomicAdd(&ctr[i], sm);
            }
        }
        const unsigned long long any = __ballot(still);
        if (lane == 0) st.tile_active[tile] = any != 0ull ? 1 : 0;
        cnt[f] = 0;
    }
    __syncthreads();  // every wave has read zt
    for (int w = wave; w < nw; w += kTailWaves) zt[w * kTile] = 0u;
}

// ------------------------------------------------------------ plumbing kernels
__global__ void reset_kernel(DevState st) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= st.ntiles * kTile) return;
    const bool valid = f < st.count;
    st.done[f] = valid ? 0 : 1;
    st.conv[f] = -1;
    st.status[f] = 1;
    st.iters[f] = 0;
    st.nllr_cnt[f] = 0;
    if ((f & 63) == 0) st.tile_active[f >> 6] = valid ? 1 : 0;
}

// Streaming Monte-Carlo: every lane empty and asking for a frame.
__global__ void stream_init_kernel(DevState st) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= st.ntiles * kTile) return;
    st.done[f] = 1;
    st.refill[f] = 1;
    st.fresh[f] = 0;
    st.iters[f] = 0;
    st.nllr_cnt[f] = 0;
    if ((f & 63) == 0) st.tile_active[f >> 6] = 0;
}

// llr [count][n] (row per frame) -> ch [tile][n][64]
__global__ void load_llr_kernel(DevGraph g, DevState st, const double *llr) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)st.ntiles * g.n * kTile;
    if (i >= total) return;
    const int lane = (int)(i & 63);
    const size_t tj = i >> 6;
    const int j = (int)(tj % g.n);
    const int tile = (int)(tj / g.n);
    const int f = tile * kTile + lane;
    st.ch[i] = f < st.count ? llr[(size_t)f * g.n + j] : 0.0;
}

// L [tile][n][64] -> z [count][n] (uint8, z = L<0) and optional post [count][n]
__global__ void finalize_kernel(DevGraph g, DevState st, uint8_t *z, double *post) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)st.count * g.n;
    if (i >= total) return;
    const int f = (int)(i / g.n);
    const int j = (int)(i % g.n);
    const double L = st.L[((size_t)(f >> 6) * g.n + j) * kTile + (f & 63)];
    z[i] = L < 0.0 ? 1 : 0;
    if (post) post[i] = L;
}

__global__ void export_msgs_kernel(DevGraph g, DevState st, double *out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)st.count * g.nnz;
    if (i >= total) return;
    const int f = (int)(i / g.nnz);
    const int e = (int)(i % g.nnz);
    out[i] = st.E[e_base(g, f >> 6, f & 63) + (size_t)e * g.ef];
}

// Streaming refill (Monte-Carlo path): every lane flagged by vn_kernel (or, at
// the start, every lane) takes the next frame index from one device counter
// (wave-aggregated atomicAdd; wave 0 of the tile's block) and the block's 8
// wavefronts generate the new frames in place (gen_slots); with no frame left
// the lane goes idle.  Lanes of one tile therefore decode different frames at
// different iterations -- each lane's state depends on its own frame only.
constexpr int kRefillThreads = 512;  // 8 wavefronts share a tile's frame generation (gen_slots)
__global__ __launch_bounds__(kRefillThreads) void refill_kernel(DevGraph g, DevState st, uint64_t seed,
                                                                int snr_point, double sigma, int64_t frame0,
                                                                int64_t total, unsigned long long *next) {
    extern __shared__ uint32_t ul[];  // [kw][64] u-bit stage
    __shared__ long long gidx[kTile];
    __shared__ int gen;
    const int tile = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int f = tile * kTile + lane;
    if (threadIdx.x < kTile) {  // wave 0: the lanes to refill take the next indices
        const bool need = st.refill[f] != 0;
        const unsigned long long want = __ballot(need);
        bool have = false;
        long long gi = -1;
        if (want != 0ull) {
            const unsigned long long below = lane ? (want & (~0ull >> (64 - lane))) : 0ull;
            unsigned long long base = 0ull;
            if (lane == __ffsll((long long)want) - 1) base = atomicAdd(next, (unsigned long long)__popcll(want));
            base = __shfl(base, __ffsll((long long)want) - 1);
            const int64_t idx = (int64_t)(base + (unsigned long long)__popcll(below));
            have = need && idx < total;
            if (have) gi = supply_frame(st, frame0, idx);
            if (need) {
                st.refill[f] = 0;
                st.done[f] = have ? 0 : 1;
                st.fresh[f] = have ? 1 : 0;
                st.iters[f] = 0;
            }
        }
        gidx[lane] = gi;
        const unsigned long long busy = __ballot(st.done[f] == 0);
        const unsigned long long took = __ballot(have);  // (a ballot of the whole wavefront)
        if (lane == 0) {
            if (want != 0ull) st.tile_active[tile] = busy != 0ull ? 1 : 0;
            gen = took != 0ull ? 1 : 0;
        }
    }
    __syncthreads();
    if (gen) gen_slots<kTile>(g, st, tile, 0, gidx, ul, seed, snr_point, sigma);
}

__global__ void export_frames_kernel(DevGraph g, DevState st, uint8_t *u_out, double *llr_out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)st.count * g.n;
    if (i >= total) return;
    const int f = (int)(i / g.n);
    const int j = (int)(i % g.n);
    const int tile = f >> 6, lane = f & 63;
    if (llr_out) llr_out[i] = st.ch[((size_t)tile * g.n + j) * kTile + lane];
    if (u_out && j < g.k) {
        const int kw = (g.k + 31) >> 5;
        const uint32_t w = st.ubits[((size_t)tile * kw + (j >> 5)) * kTile + lane];
        u_out[(size_t)f * g.k + j] = (uint8_t)((w >> (j & 31)) & 1u);
    }
}

// Per-frame Monte-Carlo counters (main.py:130-138 + :154-172), one wave per tile.
__global__ __launch_bounds__(64) void count_kernel(DevGraph g, DevState st, unsigned long long *ctr) {
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int f = tile * kTile + lane;
    const bool valid = f < st.count;
    const int kw = (g.k + 31) >> 5;
    unsigned long long v[7] = {0, 0, 0, 0, 0, 0, 0};
    if (valid) {
        const bool ok = st.status[f] == 0;
        v[0] = 1;
        v[1] = ok ? 0 : 1;
        if (!ok) {  // BER counts only frames whose syndrome check failed (main.py:130-138)
            const double *Lt = st.L + (size_t)tile * g.n * kTile + lane;
            unsigned long long err = 0;
            for (int w = 0; w < kw; ++w) {
                const uint32_t u = st.ubits[((size_t)tile * kw + w) * kTile + lane];
                uint32_t dec = 0u;
                const int nb = min(32, g.k - w * 32);
                for (int b = 0; b < nb; ++b)
                    dec |= (Lt[(w * 32 + b) * kTile] < 0.0 ? 0u : 1u) << b;  // z^1
                err += __popc(u ^ dec);
            }
            v[2] = err;
        }
        const int cv = st.conv[f];
        v[3] = cv >= 0 ? (unsigned long long)cv : 0;
        v[4] = cv >= 0 ? 1 : 0;
        v[5] = (unsigned long long)st.nllr_cnt[f];
        v[6] = (unsigned long long)st.iters[f];
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const unsigned long long s = wave_sum(v[i]);
        if (lane == 0 && s) atomicAdd(&ctr[i], s);
    }
}

inline unsigned grid_for(size_t total, int block) { return (unsigned)((total + block - 1) / block); }

}  // namespace

hipError_t launch_reset(const DevGraph &, const DevState &st, hipStream_t s) {
    const int total = st.ntiles * kTile;
    reset_kernel<<<grid_for(total, 256), 256, 0, s>>>(st);
    return hipGetLastError();
}

hipError_t launch_load_llr(const DevGraph &g, const DevState &st, const double *llr, hipStream_t s) {
    const size_t total = (size_t)st.ntiles * g.n * kTile;
    load_llr_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, llr);
    return hipGetLastError();
}

// cn_row_kernel for rows of degree <= 192; LDPC_CN_ROW=0 forces cn_kernel (A/B)
bool use_cn_row(const DevGraph &g) {
    static const int force = [] {
        const char *e = getenv("LDPC_CN_ROW");
        return e ? atoi(e) : -1;
    }();
    return force != 0 && g.max_row_deg <= kRowW * kRowK;
}

// 16 x 40 shape for rows of 193..640 edges, from 64 tiles on: on a full chunk
// of wimax_2304_0.5 (128 tiles) its CN pass is 10 % faster than cn_kernel's
// (16 B instead of 24 B per edge, one tanh per edge instead of two); in the
// few-tile streaming tail, where one 16-wavefront workgroup per CU is all
// that fits, 1.5 % slower (profiles/r2aw_cn_row16).  LDPC_CN_ROW16 (read per
// call): 0 = never, 1 = at any tile count, N > 1 = from N tiles, unset = from
// 64 tiles -- but cn_sub_kernel takes the 2304 codes up to 128 tiles first
// (use_cn_sub; round 5: equal on a 128-tile split chunk, 8 % faster in the
// 3 dB streaming tail, profiles/r5_ab/r5ad_ab), so this runs above 128.
constexpr int kRow16W = 16, kRow16K = 40;
bool use_cn_row16(const DevGraph &g, int ntiles) {
    if (use_cn_row(g) || g.max_row_deg > kRow16W * kRow16K) return false;
    const char *e = getenv("LDPC_CN_ROW16");
    const int from = e ? atoi(e) : 64;
    return from != 0 && ntiles >= from;
}

template <bool kFirst, bool kStream>
void launch_cn_row(const DevGraph &g, const DevState &st, int par, hipStream_t s) {
    const unsigned grid = (unsigned)(((st.ntiles + 7) / 8) * 8 * g.m);
    const int *ci = g.col_idx, *rp = g.row_ptr;
    if (use_cn_row(g))
        cn_row_kernel<kFirst, kStream, 4, 6><<<grid, 64 * kRowW, 0, s>>>(g, st, par, ci, rp, kAtanhCoef);
    else
        cn_row_kernel<kFirst, kStream, 4, 4, kRow16W, kRow16K><<<grid, 64 * kRow16W, 0, s>>>(g, st, par, ci, rp,
                                                                                            kAtanhCoef);
}

// cn_sub_kernel (cn_sub.hip: 16-frame sub-tiles, t in registers, one tanh per
// edge) for the long rows of the 2304 codes up to LDPC_CN_SUB tiles (read per
// call; 0 = never; default kCnSubTiles: the streaming tail and small split
// batches, where cn_kernel's two tanh per edge made it VALU-issue bound).
constexpr int kCnSubTiles = 128;
bool use_cn_sub(const DevGraph &g, int ntiles) {
    if (use_cn_row(g) || !cn_sub_shape(g)) return false;
    const char *e = getenv("LDPC_CN_SUB");
    const int lim = e ? atoi(e) : kCnSubTiles;
    return ntiles <= lim;
}

hipError_t launch_cn(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream) {
    if (use_cn_sub(g, st.ntiles)) return launch_cn_sub(g, st, it, s, stream);
    if (use_cn_row(g) || use_cn_row16(g, st.ntiles)) {
        const int par = it & 1;
        if (stream)
            launch_cn_row<false, true>(g, st, par, s);
        else if (it == 0)
            launch_cn_row<true, false>(g, st, par, s);
        else
            launch_cn_row<false, false>(g, st, par, s);
        return hipGetLastError();
    }
    const int bpt = (g.m + kCnRowsPerBlock - 1) / kCnRowsPerBlock;
    const unsigned grid = (unsigned)(((st.ntiles + 7) / 8) * 8 * bpt);
    const int par = it & 1;
    if (stream)
        cn_kernel<false, true><<<grid, 256, 0, s>>>(g, st, bpt, par, g.col_idx, g.row_ptr, kAtanhCoef);
    else if (it == 0)
        cn_kernel<true, false><<<grid, 256, 0, s>>>(g, st, bpt, par, g.col_idx, g.row_ptr, kAtanhCoef);
    else
        cn_kernel<false, false><<<grid, 256, 0, s>>>(g, st, bpt, par, g.col_idx, g.row_ptr, kAtanhCoef);
    return hipGetLastError();
}

hipError_t launch_cn_rare(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream) {
    const unsigned grid = (unsigned)(st.nslots / 4);
    const int par = it & 1;
    if (stream)
        cn_rare_kernel<false, true><<<grid, 256, 0, s>>>(g, st, par, kAtanhCoef);
    else if (it == 0)
        cn_rare_kernel<true, false><<<grid, 256, 0, s>>>(g, st, par, kAtanhCoef);
    else
        cn_rare_kernel<false, false><<<grid, 256, 0, s>>>(g, st, par, kAtanhCoef);
    return hipGetLastError();
}

hipError_t launch_vn(const DevGraph &g, const DevState &st, int it, int max_iter, bool nllr, hipStream_t s,
                     unsigned long long *stream_ctr) {
    const size_t lds = (size_t)((g.m + 31) >> 5) * kTile * sizeof(uint32_t);
    const int last = it == max_iter - 1 ? 1 : 0;
    const int nl = nllr ? 1 : 0;
    if (stream_ctr)
        vn_kernel<false, true><<<st.ntiles, kVnWaves * 64, lds, s>>>(g, st, it, max_iter, nl, g.csc_ptr,
                                                                      g.csc_edge, g.csc_row, stream_ctr);
    else if (it == 0)
        vn_kernel<true, false><<<st.ntiles, kVnWaves * 64, lds, s>>>(g, st, it, last, nl, g.csc_ptr, g.csc_edge,
                                                                      g.csc_row, nullptr);
    else
        vn_kernel<false, false><<<st.ntiles, kVnWaves * 64, lds, s>>>(g, st, it, last, nl, g.csc_ptr, g.csc_edge,
                                                                       g.csc_row, nullptr);
    return hipGetLastError();
}

hipError_t launch_vn_tail(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint32_t *zb, int *cnt,
                          unsigned long long *ctr, hipStream_t s) {
    if (!g.a_packed || !st.ubits || ((g.k + 31) >> 5) > kTailKw) return hipErrorInvalidValue;
    vn_cols_kernel<<<dim3((unsigned)((g.n + 3) / 4), (unsigned)st.ntiles), 256, 0, s>>>(g, st, nllr ? 1 : 0, zb, cnt,
                                                                                      0);
    tail_exit_kernel<false><<<st.ntiles, 64 * kTailWaves, 0, s>>>(g, st, 0, max_iter, nllr ? 1 : 0, zb, cnt, ctr,
                                                                  nullptr);
    return hipGetLastError();
}

// ldpc_decode_f64 on few tiles: pass `it` of the column-parallel VN
hipError_t launch_vn_cols_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                 int *cnt, hipStream_t s) {
    if (!g.a_packed || ((g.k + 31) >> 5) > kTailKw) return hipErrorInvalidValue;
    vn_cols_kernel<<<dim3((unsigned)((g.n + 3) / 4), (unsigned)st.ntiles), 256, 0, s>>>(g, st, nllr ? 1 : 0, zb, cnt,
                                                                                      it == 0 ? 1 : 0);
    return launch_tail_exit_decode(g, st, it, last, nllr, zb, cnt, nullptr, s);
}

hipError_t launch_tail_exit_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                   int *cnt, int *gbad, hipStream_t s) {
    tail_exit_kernel<true><<<st.ntiles, 64 * kTailWaves, 0, s>>>(g, st, it, last ? 1 : 0, nllr ? 1 : 0, zb, cnt,
                                                                 nullptr, gbad);
    return hipGetLastError();
}

hipError_t launch_stream_init(const DevGraph &, const DevState &st, hipStream_t s) {
    const int total = st.ntiles * kTile;
    stream_init_kernel<<<grid_for(total, 256), 256, 0, s>>>(st);
    return hipGetLastError();
}

hipError_t launch_refill(const DevGraph &g, const DevState &st, uint64_t seed, int snr_point, double sigma,
                         int64_t frame0, int64_t total, unsigned long long *next, hipStream_t s) {
    const size_t lds = (size_t)((g.k + 31) >> 5) * kTile * sizeof(uint32_t);
    refill_kernel<<<st.ntiles, kRefillThreads, lds, s>>>(g, st, seed, snr_point, sigma, frame0, total, next);
    return hipGetLastError();
}

// ------------------------------------------------ streaming tail compaction
// Once the frame supply is out, the frames still running are scattered over
// every tile and each step still costs every tile they touch.  Frames running
// in tiles >= nt move into finished slots of tiles < nt (sources and
// destinations are disjoint: no ordering hazard); the steps after that launch
// nt tiles.  A frame's state is its lane of E, L, ch, ubits and its iters /
// fresh flags -- it decodes exactly as before, so the counters do not change.
// plan (one workgroup): pairs[0] = P, pairs[1..P] sources, pairs[1+cap..] destinations
__global__ __launch_bounds__(1024) void compact_plan_kernel(DevState st, int nt, int cap, int *pairs) {
    __shared__ int sa[1024], sb[1024];
    const int slots = st.ntiles * kTile, low = nt * kTile;
    const int per = (slots + blockDim.x - 1) / blockDim.x;
    const int b0 = threadIdx.x * per, b1 = min(slots, b0 + per);
    int na = 0, nb = 0;  // live in the high tiles, finished in the low tiles
    for (int f = b0; f < b1; ++f) {
        const bool live = st.done[f] == 0;
        na += (f >= low && live) ? 1 : 0;
        nb += (f < low && !live) ? 1 : 0;
    }
    sa[threadIdx.x] = na;
    sb[threadIdx.x] = nb;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {  // inclusive scans
        const int va = threadIdx.x >= (unsigned)o ? sa[threadIdx.x - o] : 0;
        const int vb = threadIdx.x >= (unsigned)o ? sb[threadIdx.x - o] : 0;
        __syncthreads();
        sa[threadIdx.x] += va;
        sb[threadIdx.x] += vb;
        __syncthreads();
    }
    int ia = sa[threadIdx.x] - na, ib = sb[threadIdx.x] - nb;
    const int P = min(sa[blockDim.x - 1], sb[blockDim.x - 1]);
    for (int f = b0; f < b1; ++f) {
        const bool live = st.done[f] == 0;
        if (f >= low && live) {
            if (ia < P) pairs[1 + ia] = f;
            ++ia;
        } else if (f < low && !live) {
            if (ib < P) pairs[1 + cap + ib] = f;
            ++ib;
        }
    }
    if (threadIdx.x == 0) pairs[0] = P;
}

// move: every (item, pair) of E / L / ch / ubits.  Pair-fastest: the plan
// lists sources and destinations in ascending slot order, so consecutive
// threads move neighbouring lanes of one item (the lanes of a 512 B row),
// not one lane's items 512 B apart.
__global__ void compact_move_kernel(DevGraph g, DevState st, int cap, const int *pairs) {
    const int P = pairs[0];
    const int kw = (g.k + 31) >> 5;
    const int64_t items = (int64_t)g.nnz + 2 * (int64_t)g.n + kw;
    const int64_t total = (int64_t)P * items;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i % P);
        int64_t it = i / P;
        const int src = pairs[1 + p], dst = pairs[1 + cap + p];
        const size_t st_ = src >> 6, sl = src & 63, dt = dst >> 6, dl = dst & 63;
        if (it < g.nnz) {
            st.E[e_base(g, (int)dt, (int)dl) + (size_t)it * g.ef] = st.E[e_base(g, (int)st_, (int)sl) + (size_t)it * g.ef];
            continue;
        }
        it -= g.nnz;
        if (it < g.n) {
            st.L[(dt * g.n + it) * kTile + dl] = st.L[(st_ * g.n + it) * kTile + sl];
            continue;
        }
        it -= g.n;
        if (it < g.n) {
            st.ch[(dt * g.n + it) * kTile + dl] = st.ch[(st_ * g.n + it) * kTile + sl];
            continue;
        }
        it -= g.n;
        st.ubits[(dt * kw + it) * kTile + dl] = st.ubits[(st_ * kw + it) * kTile + sl];
    }
}

__global__ void compact_flags_kernel(DevState st, int cap, const int *pairs) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= pairs[0]) return;
    const int src = pairs[1 + p], dst = pairs[1 + cap + p];
    st.done[dst] = 0;
    st.refill[dst] = 0;
    st.iters[dst] = st.iters[src];
    st.fresh[dst] = st.fresh[src];
    st.done[src] = 1;
    st.refill[src] = 0;
    st.fresh[src] = 0;
}

__global__ void tile_active_kernel(DevState st) {  // after a compaction: which of the nt tiles run
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const unsigned long long busy = __ballot(st.done[tile * kTile + lane] == 0);
    if (lane == 0) st.tile_active[tile] = busy != 0ull ? 1 : 0;
}

hipError_t launch_compact_plan(const DevState &st, int nt, int cap, int *pairs, hipStream_t s) {
    compact_plan_kernel<<<1, 1024, 0, s>>>(st, nt, cap, pairs);
    return hipGetLastError();
}

hipError_t launch_compact(const DevGraph &g, const DevState &st, int nt, int cap, int *pairs, hipStream_t s) {
    compact_plan_kernel<<<1, 1024, 0, s>>>(st, nt, cap, pairs);
    compact_move_kernel<<<2048, 256, 0, s>>>(g, st, cap, pairs);
    compact_flags_kernel<<<grid_for(cap, 256), 256, 0, s>>>(st, cap, pairs);
    DevState lo = st;
    lo.ntiles = nt;
    tile_active_kernel<<<nt, kTile, 0, s>>>(lo);
    return hipGetLastError();
}

hipError_t launch_finalize(const DevGraph &g, const DevState &st, uint8_t *z, double *post, hipStream_t s) {
    const size_t total = (size_t)st.count * g.n;
    if (total) finalize_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, z, post);
    return hipGetLastError();
}

hipError_t launch_export_msgs(const DevGraph &g, const DevState &st, double *out, hipStream_t s) {
    const size_t total = (size_t)st.count * g.nnz;
    if (total) export_msgs_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, out);
    return hipGetLastError();
}

hipError_t launch_export_frames(const DevGraph &g, const DevState &st, uint8_t *u_out, double *llr_out,
                                hipStream_t s) {
    const size_t total = (size_t)st.count * g.n;
    if (total) export_frames_kernel<<<grid_for(total, 256), 256, 0, s>>>(g, st, u_out, llr_out);
    return hipGetLastError();
}

hipError_t launch_count(const DevGraph &g, const DevState &st, unsigned long long *counters, hipStream_t s) {
    count_kernel<<<st.ntiles, kTile, 0, s>>>(g, st, counters);
    return hipGetLastError();
}

}  // namespace ldpc
