// tile_kernels.hip -- the tile-resident parity decoder (gfx950).
//
// One workgroup (16 wavefronts, lane = frame) decodes one tile of 64 frames
// through ALL its iterations of python_ldpc_app/spa_decoder.py:104-276, with
// the check-node update (:112-168), the variable-node sum (:173-185), the hard
// decision / syndrome / early termination (:188-253) and the M update
// (:260-268) in one launch.  For graphs H_std = [A | I_m] whose column sums of
// the A part fit in LDS (k x 64 frames x 8 B: wimax_576_0.5, k = 288 ->
// 144 KB), the variable-node pass needs no second sweep over E:
//
//   rows are processed in ascending order, so the sum of column j,
//   S_j = ((0 + E_r0j) + E_r1j) + ...  rows ascending (scipy csr_matvec of
//   E^T, the reference's rounding order), is accumulated in LDS as each row's
//   new messages are produced.  Identity column k+r has one edge (row r):
//   its posterior ch + (0 + E) is final when row r is.
//
// HBM traffic per edge and iteration is the algorithmic 16 B (E_old read +
// E_new write) plus the posterior gather L[col] (served by L2/MALL: a tile's
// L is 295 KB); the separate CN/VN launches move 24 B + the gather.
//
// Within a row (degree <= 192) wavefront w owns the contiguous chunk of
// C = ceil(deg/16) edges starting at position w*C and keeps their t in
// registers.  P = t0*t1*... is formed strictly left to right by handing the
// running product from wavefront to wavefront through an LDS slot guarded by
// an epoch-tagged flag (no workgroup barrier).  Each wavefront runs the
// software pipeline
//
//   body(r):  P3(r-1)  E_new = 2 atanh(clip(P/t)) of its chunk of row r-1,
//                      stores E_new, adds it into S (or writes the identity
//                      column's posterior);
//             hop(r)   waits for wavefront w-1's product of row r, multiplies
//                      its chunk in, publishes;
//             P1(r+1)  loads L[col] and E_old of its chunk of row r+1,
//                      t = tanh((L - E_old)/2).
//
// Ordering of the S additions: any P3(r) waits for the final product of row r,
// published by the last hop(r); every wavefront's hop(r) follows its own
// P3(r-1) in program order, so all additions of row r-1 precede any of row r
// (a column occurs once per row, so no two additions of one row collide).
// The same argument lets two chain slots serve all rows.
//
// Rare rows (some |t| <= 1e-10, spa_decoder.py:159-164): every wavefront parks
// its t in the workgroup's scratch slot (global, read back through L2) and
// the "product of the others" is walked there.
//
// End of a pass: L_j = ch_j + S_j for the A columns (the normalized-LLR count
// :210-228 against the previous posterior), the z^1 bit vectors of all
// columns in LDS, one sweep over the rows for the syndrome, and the per-frame
// exit decisions of vn_kernel (static schedule).  The tile stops when none of
// its frames is running.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "cn_common.h"
#include "tile_common.h"
#include "spa_device.h"
#include "spa_math.h"
#include "frame_source.h"

namespace ldpc {
namespace {

constexpr int kTW = 16;               // wavefronts per workgroup
constexpr int kTK = 192 / kTW;        // edges per wavefront chunk: row degree <= kTW * kTK = 192
constexpr int kTR = 2;                // chain slots (see the ordering argument above)
constexpr size_t kTileLdsMax = 163840;
constexpr int kTKW = 10;  // (z^1)_A words per lane held in registers for the syndrome: k <= 320

// Dynamic LDS carve (bytes); every region 16-B aligned.
struct TileLayout {
    size_t S, math, slot, zb, ib, lane_i, flags, total;
};
__host__ __device__ inline TileLayout tile_layout(int k, int m) {
    TileLayout t;
    size_t o = 0;
    t.S = o;
    o = al16(o + (size_t)k * kTile * sizeof(double));
    t.math = o;
    o = al16(o + sizeof(MathLds));
    t.slot = o;
    o = al16(o + (size_t)kTR * kTile * sizeof(double));
    t.zb = o;
    o = al16(o + (size_t)((k + 31) / 32) * kTile * sizeof(uint32_t));
    t.ib = o;
    o = al16(o + (size_t)((m + 31) / 32) * kTile * sizeof(uint32_t));
    t.lane_i = o;  // bad[64], nllr count[64], live[64]
    o = al16(o + 3 * kTile * sizeof(int));
    t.flags = o;  // chain flag[kTR], tiny[kTR], tiny sequence, tile running
    o = al16(o + (2 * kTR + 2) * sizeof(int));
    t.total = o;
    return t;
}

// The message stream (E_old loads, E_new stores) is non-temporal: read once and
// written once per pass, it then does not evict the tile's posteriors (the
// L[col] gather) from L2 (profiles/r1u_nt).
__device__ __forceinline__ double ld_msg(const double *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_msg(double *p, double v) { __builtin_nontemporal_store(v, p); }

// element (item, lane) of a tile array
template <class T>
__device__ __forceinline__ T *at(T *base, int item, uint32_t lane) {
    return base + (size_t)item * kTile + lane;
}

struct RowChunk {
    int beg, deg, C, c0, cnt;
};
__device__ __forceinline__ RowChunk chunk_of(const int *__restrict__ row_ptr, int r, int wave) {
    RowChunk c;
    c.beg = row_ptr[r];
    c.deg = row_ptr[r + 1] - c.beg;
    c.C = (c.deg + kTW - 1) / kTW;
    c.c0 = c.beg + wave * c.C;
    c.cnt = max(0, min(c.deg - wave * c.C, c.C));
    return c;
}

struct TileCtx {
    const int *__restrict__ col_idx;
    const int *__restrict__ row_ptr;
    // tile bases (uniform); element (item, lane) at [item * 64 + lane]
    double *Eb;        // messages E
    double *Lb;        // posteriors
    const double *Cb;  // channel LLRs
    double *Tb;        // rare-row scratch slot of this workgroup: two buffers, by rare-row parity
    size_t tbuf;       // doubles between the two buffers
    double *S;         // LDS [k][64]
    double *slot;      // LDS [kTR][64]
    uint32_t *ib;      // LDS [mw][64] z^1 of the identity columns
    int *flag, *tinyf, *tseq;
    LdsTanh ttab;
    LdsAtanh ltab;
    AtanhCoef ac;   // kernel-argument coefficients (when coef_arg)
    bool coef_arg;  // P3 uses ac instead of coef_load() (compile-time per kernel)
    int k, wave;
    uint32_t lane;
    int ep0;  // epoch of row 0 in this pass (flags are tagged (epoch, stage))
    bool first, live;
    bool fresh;  // streaming: this lane's frame is on its first pass (M = L - 0)
    int ntiny;
};

// P1 pieces: L[col] of edge i of chunk rc, E_old, and t = tanh((L - E_old)/2).
// Loads are unconditional (index clamped into the chunk).
__device__ __forceinline__ double tile_load_l(const TileCtx &c, const RowChunk &rc, int i) {
    const double *Ls = c.first ? c.Cb : c.Lb;
    return ld_l2(at(Ls, c.col_idx[rc.c0 + min(i, rc.cnt - 1)], c.lane));
}
__device__ __forceinline__ double tile_load_e(const TileCtx &c, const RowChunk &rc, int i) {
    return c.first ? 0.0 : ld_msg(at(c.Eb, rc.c0 + min(i, rc.cnt - 1), c.lane));
}
__device__ __forceinline__ bool tile_t(const TileCtx &c, double &t, double eo) {
    const double M = c.first ? t : t - (c.fresh ? 0.0 : eo);  // :85-90 / :260-268
    // tanh evaluated for every lane, the +-17.5 clip on the output (the
    // clamped-input form, tanh_half_clipped, spills here and measured 26 %
    // slower on wimax_576_0.5)
    t = clip_cl(np_tanh(M * 0.5, c.ttab));  // :138-146 (tests/test_math.py: output clip == input clip)
    return c.live && !(fabs(t) > kTiny);  // a frame-less lane never votes
}

// P1: loads of the chunk, then t = tanh((L - E_old)/2) edge by edge; returns
// whether some lane has |t| <= 1e-10.
__device__ __forceinline__ bool tile_p1(const TileCtx &c, const RowChunk &rc, double (&t)[kTK]) {
    bool tiny = false;
    if (rc.cnt > 0) {
        double eo[kTK];
#pragma unroll
        for (int i = 0; i < kTK; ++i) {
            if (i < rc.cnt) {
                t[i] = tile_load_l(c, rc, i);
                eo[i] = tile_load_e(c, rc, i);
            }
        }
#pragma unroll
        for (int i = 0; i < kTK; ++i)
            if (i < rc.cnt) tiny |= tile_t(c, t[i], eo[i]);
    }
    return __ballot(tiny) != 0ull;
}

// P * t[0] * t[1] * ... * t[cnt-1], left to right, as exactly cnt dependent
// multiplies: one uniform branch on cnt selects a straight-line sequence (a
// guarded loop was if-converted into mul + 2 v_cndmask per slot for all kTK
// slots -- 3x the dependent chain on the row's critical path).
template <int N>
__device__ __forceinline__ double mul_n(double P, const double (&t)[kTK]) {
#pragma unroll
    for (int i = 0; i < N; ++i) P = P * t[i];
    return P;
}
template <int N>
struct ChainMul {
    static __device__ __forceinline__ double run(double P, const double (&t)[kTK], int cnt) {
        if (cnt == N) return mul_n<N>(P, t);
        return ChainMul<N - 1>::run(P, t, cnt);
    }
};
template <>
struct ChainMul<0> {
    static __device__ __forceinline__ double run(double P, const double (&)[kTK], int) { return P; }
};

// hop: this wavefront's segment of row r's left-to-right product.
__device__ __forceinline__ void tile_hop(const TileCtx &c, int r, const double (&t)[kTK], bool tiny) {
    const RowChunk rc = chunk_of(c.row_ptr, r, c.wave);
    if (rc.deg == 0) return;  // spa_decoder.py:115-122
    const int s = r & (kTR - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    double *sl = c.slot + s * kTile + c.lane;
    double P;
    if (c.wave == 0) {
        P = ChainMul<kTK>::run(1.0, t, rc.cnt);  // 1.0 * t0 == t0 exactly
        if (c.lane == 0) lds_st(c.tinyf + s, tiny ? 1 : 0);
    } else {
        wait_flag(c.flag + s, ep + c.wave);
        P = ChainMul<kTK>::run(*sl, t, rc.cnt);
        if (tiny && c.lane == 0) lds_st(c.tinyf + s, 1);
    }
    *sl = P;
    lds_release();
    if (c.lane == 0) lds_st(c.flag + s, ep + c.wave + 1);
}

// P3: E_new of this wavefront's chunk of row r, stored and folded into the
// column sums (t is overwritten with E_new).
__device__ __forceinline__ void tile_p3(TileCtx &c, int r, double (&t)[kTK]) {
    const RowChunk rc = chunk_of(c.row_ptr, r, c.wave);
    if (rc.deg == 0) return;
    const int s = r & (kTR - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    wait_flag(c.flag + s, ep + kTW);
    const double P = c.slot[s * kTile + c.lane];
    const bool tiny_row = uniform(lds_ld(c.tinyf + s)) != 0;
    const AtanhCoef ac = c.coef_arg ? c.ac : coef_load();  // scalar loads for this P3 only (cn_common.h)
    if (!tiny_row) {
#pragma unroll
        for (int i = 0; i < kTK; ++i)
            if (i < rc.cnt) t[i] = 2.0 * atanh_f(clip_cl(P / t[i]), c.ltab, ac);  // :159-168
    } else {
        // rare: q = prod of the others, in order (np.prod(np.delete(...)), :164)
        // the rare rows alternate between two scratch buffers: a wavefront
        // parks the next rare row's t only after every wavefront has counted
        // that row, i.e. finished reading this one
        double *tb = c.Tb + (c.ntiny & 1) * c.tbuf;
        const int pos0 = c.wave * rc.C;
#pragma unroll
        for (int i = 0; i < kTK; ++i)
            if (i < rc.cnt) *at(tb, pos0 + i, c.lane) = t[i];
        __builtin_amdgcn_s_waitcnt(0);  // scratch stores have reached L2
        c.ntiny += 1;
        if (c.lane == 0) __hip_atomic_fetch_add(c.tseq, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_flag(c.tseq, c.ntiny * kTW);
#pragma unroll
        for (int i = 0; i < kTK; ++i) {
            if (i < rc.cnt) {
                const double ti = t[i];
                double q;
                if (fabs(ti) > kTiny) {
                    q = P / ti;
                } else {
                    q = 1.0;
                    bool fst = true;
                    for (int p = 0; p < rc.deg; ++p) {
                        if (p == pos0 + i) continue;
                        const double t2 = ld_l2(at(tb, p, c.lane));
                        q = fst ? t2 : q * t2;
                        fst = false;
                    }
                }
                t[i] = 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
            }
        }
    }
    if (c.live) {  // the chunk's E_new stores under ONE exec mask
#pragma unroll
        for (int i = 0; i < kTK; ++i)
            if (i < rc.cnt) st_msg(at(c.Eb, rc.c0 + i, c.lane), t[i]);
    }
#pragma unroll
    for (int i = 0; i < kTK; ++i) {
        if (i < rc.cnt) {
            const int col = c.col_idx[rc.c0 + i];
            if (col < c.k) {  // S_col += E (rows ascending)
                double *sp = c.S + col * kTile + c.lane;
                // one ds_add_f64: the same IEEE add as read / add / write (tile_sub.hip)
                __hip_atomic_fetch_add(sp, t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {  // identity column: L = ch + (0 + E)  (:173-185)
                const double Lj = *at(c.Cb, col, c.lane) + (0.0 + t[i]);
                if (c.live) *at(c.Lb, col, c.lane) = Lj;
                if (!(Lj < 0.0)) {
                    const int q = col - c.k;
                    atomicOr(c.ib + (q >> 5) * kTile + c.lane, 1u << (q & 31));
                }
            }
        }
    }
}

// body(r) = P3(r-1), hop(r), P1(r+1)
__device__ __forceinline__ void tile_body(TileCtx &c, int r, int m, double (&tcur)[kTK], bool &ycur,
                                          double (&toth)[kTK], bool &yoth) {
    RowChunk rc1{};
    if (r + 1 < m) rc1 = chunk_of(c.row_ptr, r + 1, c.wave);
    if (r >= 1) tile_p3(c, r - 1, toth);
    if (r < m) tile_hop(c, r, tcur, ycur);
    if (r + 1 < m) yoth = tile_p1(c, rc1, toth);
}

// End of a pass, once every column's z^1 bit is in zb (A part) / ib (identity
// part) and the normalized-LLR counts are in cntl: the syndrome (:191-204) of
// every frame and the per-frame exits of vn_kernel (static schedule).  Row r
// of H_std = [A | I] has parity popcount(A_r & (z^1)_A) + (z^1)_{k+r}; A_r is
// bit-packed (g.a_packed, scalar loads), this lane's (z^1)_A words sit in
// registers.  Returns whether any frame of the tile still runs (uniform).
__device__ __forceinline__ bool tile_pass_end(const DevGraph &g, const DevState &st, uint32_t *zb, const uint32_t *ib,
                                              int *bad, int *cntl, int *livel, int *running, int it, int max_iter,
                                              int nllr, int tile, int wave, int nwaves, bool live) {
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int lane = threadIdx.x & 63;
    const int f = tile * kTile + lane;
    uint32_t acc = 0u;
    {
        uint32_t zr[kTKW];
#pragma unroll
        for (int w = 0; w < kTKW; ++w) zr[w] = w < kw ? zb[w * kTile + lane] : 0u;
        for (int r = wave; r < g.m; r += nwaves) {
            const uint32_t *ar = g.a_packed + (size_t)r * kw;
            uint32_t par = ib[(r >> 5) * kTile + lane] >> (r & 31);
#pragma unroll
            for (int w = 0; w < kTKW; ++w)
                if (w < kw) par += __builtin_popcount(ar[w] & zr[w]);
            acc |= par & 1u;
        }
    }
    if (acc) atomicOr((uint32_t *)bad + lane, 1u);
    __syncthreads();

    if (wave == 0) {  // per-frame exits, as vn_kernel (static schedule)
        bool still = false;
        if (live) {
            if (nllr) {
                const int cn = cntl[lane];
                st.nllr_cnt[f] = cn;
                if (st.nllr_hist) st.nllr_hist[(size_t)f * st.hist_stride + it] = g.k > 0 ? (double)cn / g.k : 0.0;
            }
            if (bad[lane] == 0) {  // syndrome zero: Result.OK at this iteration (:231-241)
                st.done[f] = 1;
                st.conv[f] = it;
                st.status[f] = 0;
                st.iters[f] = it + 1;
            } else if (it == max_iter - 1) {  // Result.DATA_TRANSFER_NOT_OK (:244-253)
                st.done[f] = 1;
                st.conv[f] = -1;
                st.status[f] = 1;
                st.iters[f] = it + 1;
            } else {
                still = true;
            }
        }
        livel[lane] = still ? 1 : 0;
        bad[lane] = 0;
        cntl[lane] = 0;
        const unsigned long long any = __ballot(still);
        if (lane == 0) {
            *running = any != 0ull ? 1 : 0;
            if (!any) st.tile_active[tile] = 0;
        }
    }
    for (int i = threadIdx.x; i < (kw + mw) * kTile; i += blockDim.x) zb[i] = 0u;  // zb and ib are adjacent
    __syncthreads();
    return *running != 0;
}

__global__ __launch_bounds__(64 * kTW, 1) void tile_kernel(DevGraph g, DevState st, int max_iter, int nllr,
                                                           const int *__restrict__ col_idx,
                                                           const int *__restrict__ row_ptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const TileLayout ly = tile_layout(g.k, g.m);
    double *S = (double *)(lds + ly.S);
    MathLds &mlds = *(MathLds *)(lds + ly.math);
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + kTile;
    int *livel = cntl + kTile;
    int *flags = (int *)(lds + ly.flags);
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(mlds);
    for (int i = threadIdx.x; i < g.k * kTile; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * kTile; i += blockDim.x) zb[i] = 0u;  // zb and ib are adjacent
    for (int i = threadIdx.x; i < 2 * kTile; i += blockDim.x) bad[i] = 0;
    if (threadIdx.x < 2 * kTR) flags[threadIdx.x] = -1;
    if (threadIdx.x == 2 * kTR) flags[2 * kTR] = 0;
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    const int f = tile * kTile + lane;
    if (wave == 0) livel[lane] = st.done[f] == 0 ? 1 : 0;
    __syncthreads();
    if (!st.tile_active[tile]) return;

    TileCtx c;
    c.col_idx = col_idx;
    c.row_ptr = row_ptr;
    c.Eb = st.E + (size_t)tile * g.nnz * kTile;
    c.Lb = st.L + (size_t)tile * g.n * kTile;
    c.Cb = st.ch + (size_t)tile * g.n * kTile;
    c.Tb = st.T + (size_t)blockIdx.x * 2 * g.max_row_deg * kTile;
    c.tbuf = (size_t)g.max_row_deg * kTile;
    c.S = S;
    c.slot = (double *)(lds + ly.slot);
    c.ib = ib;
    c.flag = flags;
    c.tinyf = flags + kTR;
    c.tseq = flags + 2 * kTR;
    c.ttab = LdsTanh{mlds.tanh};
    c.ltab = LdsAtanh{mlds.atanh};
    c.coef_arg = false;  // the static decoder loads them
    c.k = g.k;
    c.lane = lane;
    c.wave = wave;
    c.ntiny = 0;
    c.fresh = false;
    const int m = g.m;

    for (int it = 0; it < max_iter; ++it) {
        c.first = it == 0;
        c.live = livel[lane] != 0;
        c.ep0 = it * m;
        double tA[kTK], tB[kTK];
        bool yA = false, yB = false;
        if (m > 0) yA = tile_p1(c, chunk_of(row_ptr, 0, wave), tA);
        for (int r = 0; r <= m; r += 2) {
            tile_body(c, r, m, tA, yA, tB, yB);
            if (r + 1 <= m) tile_body(c, r + 1, m, tB, yB, tA, yA);
        }
        __syncthreads();  // every P3 done: S complete, identity bits set

        // posteriors of the A columns, normalized-LLR count, z^1 bits
        int my_cnt = 0;
        for (int j = wave; j < g.k; j += kTW) {
            double *sp = S + j * kTile + lane;
            const double Sj = *sp;
            *sp = 0.0;
            const double chj = *at(c.Cb, j, lane);
            const double Lj = chj + Sj;  // channel added after the sum (:173,185)
            if (nllr) {
                const double ap = c.first ? chj : ld_l2(at(c.Lb, j, lane));  // a-priori = previous L (:274)
                my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
            }
            if (c.live) *at(c.Lb, j, lane) = Lj;
            if (!(Lj < 0.0)) atomicOr(zb + (j >> 5) * kTile + lane, 1u << (j & 31));
        }
        if (nllr && my_cnt) atomicAdd(cntl + lane, my_cnt);
        __syncthreads();

        if (!tile_pass_end(g, st, zb, ib, bad, cntl, livel, flags + 2 * kTR + 1, it, max_iter, nllr, tile, wave,
                           kTW, c.live))
            break;
    }
    count_rare_rows(st, c.tseq, kTW);
}



// ---------------------------------------------------------------------------
// Streaming tile decoder (Monte-Carlo, tile_stream_kernel).  With the static
// schedule a tile runs until its slowest frame stops: at 3 dB on wimax_576_0.5
// (2.9 iterations on average, FER 1.9 %) most tiles hold a 50-iteration frame,
// so the step costs nearly 50 passes.  Here every lane is a slot at its own
// iteration: after each pass a lane whose frame stopped adds that frame's
// counters (count_kernel's definitions, main.py:130-138) and takes the next
// frame index from one device counter; the frame is generated in place
// (gen_slots: ch and L = ch, so the next pass forms M = L - 0, its iteration
// 0).  Every frame is decoded exactly as in the static schedule (the lane's
// state depends on its own frame only), so the counters are identical.  The
// workgroup exits once the supply is exhausted and its lanes have drained.
// wave 0 of the streaming kernel: lanes with `want` take the next frame
// indices (one wave-aggregated atomicAdd) into gidx; the whole workgroup then
// generates them (frame_source.h gen_slots).  -> some lane took a frame.
__device__ __forceinline__ bool tile_refill(const DevState &st, int lane, bool want, int64_t frame0, int64_t total,
                                           unsigned long long *next, long long *gidx, int *livel, int *freshl,
                                           int *itl) {
    const unsigned long long w = __ballot(want);
    const int first = __ffsll((long long)w) - 1;
    unsigned long long base = 0ull;
    if (lane == first) base = atomicAdd(next, (unsigned long long)__popcll(w));
    base = __shfl(base, first);
    const unsigned long long below = lane ? (w & (~0ull >> (64 - lane))) : 0ull;
    const int64_t idx = (int64_t)(base + (unsigned long long)__popcll(below));
    const bool have = want && idx < total;
    gidx[lane] = have ? supply_frame(st, frame0, idx) : -1ll;
    if (want) {
        livel[lane] = have ? 1 : 0;
        freshl[lane] = have ? 1 : 0;
        itl[lane] = 0;
    }
    return __ballot(have) != 0ull;
}

__global__ __launch_bounds__(64 * kTW, 1) void tile_stream_kernel(DevGraph g, DevState st, int max_iter, int nllr,
                                                                  const int *__restrict__ col_idx,
                                                                  const int *__restrict__ row_ptr, AtanhCoef ac,
                                                                  uint64_t seed, int snr_point, double sigma,
                                                                  int64_t frame0, int64_t total,
                                                                  unsigned long long *next,
                                                                  unsigned long long *ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const TileLayout ly = tile_layout(g.k, g.m);
    double *S = (double *)(lds + ly.S);
    MathLds &mlds = *(MathLds *)(lds + ly.math);
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + kTile;
    int *livel = cntl + kTile;
    int *flags = (int *)(lds + ly.flags);
    __shared__ int itl[kTile], freshl[kTile];
    __shared__ long long gidx[kTile];  // refill: lane's new frame index (< 0: none)
    __shared__ int nref;               // refill: some lane took a frame this pass
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(mlds);
    for (int i = threadIdx.x; i < g.k * kTile; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * kTile; i += blockDim.x) zb[i] = 0u;
    for (int i = threadIdx.x; i < 2 * kTile; i += blockDim.x) bad[i] = 0;
    if (threadIdx.x < 2 * kTR) flags[threadIdx.x] = -1;
    if (threadIdx.x == 2 * kTR) flags[2 * kTR] = 0;
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    bool want = true;  // wave 0: this lane asks for a frame
    if (wave == 0) {
        livel[lane] = 0;
        itl[lane] = 0;
        freshl[lane] = 0;
    }

    TileCtx c;
    c.col_idx = col_idx;
    c.row_ptr = row_ptr;
    c.Eb = st.E + (size_t)tile * g.nnz * kTile;
    c.Lb = st.L + (size_t)tile * g.n * kTile;
    c.Cb = st.ch + (size_t)tile * g.n * kTile;
    c.Tb = st.T + (size_t)blockIdx.x * 2 * g.max_row_deg * kTile;
    c.tbuf = (size_t)g.max_row_deg * kTile;
    c.S = S;
    c.slot = (double *)(lds + ly.slot);
    c.ib = ib;
    c.flag = flags;
    c.tinyf = flags + kTR;
    c.tseq = flags + 2 * kTR;
    c.ttab = LdsTanh{mlds.tanh};
    c.ltab = LdsAtanh{mlds.atanh};
    c.coef_arg = kStreamCoefArg;
    c.ac = ac;
    c.k = g.k;
    c.lane = lane;
    c.wave = wave;
    c.ntiny = 0;
    c.first = false;
    const int m = g.m;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane;

    for (int pass = 0;; ++pass) {
        // refill: lanes without a frame take the next indices (wave 0), and
        // the whole workgroup generates them (u bits staged in zb, which still
        // holds the last pass's z^1 bits: gen_slots writes a refilled lane's
        // words before reading them and clears zb; without a refill it is
        // cleared here)
        if (wave == 0) {
            bool gen = false;
            if (__ballot(want) != 0ull) gen = tile_refill(st, lane, want, frame0, total, next, gidx, livel, freshl, itl);
            want = false;
            const unsigned long long any = __ballot(livel[lane] != 0);
            if (lane == 0) {
                flags[2 * kTR + 1] = any != 0ull ? 1 : 0;
                nref = gen ? 1 : 0;
            }
        }
        __syncthreads();
        if (!flags[2 * kTR + 1]) break;  // supply exhausted, every lane drained
        if (nref)
            gen_slots<kTile>(g, st, tile, 0, gidx, zb, seed, snr_point, sigma);
        else
            for (int i = threadIdx.x; i < kw * kTile; i += blockDim.x) zb[i] = 0u;
        __syncthreads();

        c.live = livel[lane] != 0;
        c.fresh = freshl[lane] != 0;
        c.ep0 = pass * m;
        double tA[kTK], tB[kTK];
        bool yA = false, yB = false;
        if (m > 0) yA = tile_p1(c, chunk_of(row_ptr, 0, wave), tA);
        for (int r = 0; r <= m; r += 2) {
            tile_body(c, r, m, tA, yA, tB, yB);
            if (r + 1 <= m) tile_body(c, r + 1, m, tB, yB, tA, yA);
        }
        __syncthreads();

        int my_cnt = 0;
        for (int j = wave; j < g.k; j += kTW) {
            double *sp = S + j * kTile + lane;
            const double Sj = *sp;
            *sp = 0.0;
            const double chj = *at(c.Cb, j, lane);
            const double Lj = chj + Sj;  // channel added after the sum (:173,185)
            if (nllr) {
                const double ap = ld_l2(at(c.Lb, j, lane));  // previous L (= ch on a frame's first pass)
                my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
            }
            if (c.live) *at(c.Lb, j, lane) = Lj;
            if (!(Lj < 0.0)) atomicOr(zb + (j >> 5) * kTile + lane, 1u << (j & 31));
        }
        if (nllr && my_cnt) atomicAdd(cntl + lane, my_cnt);
        __syncthreads();

        // syndrome (:191-204), as tile_pass_end
        uint32_t acc = 0u;
        {
            uint32_t zr[kTKW];
#pragma unroll
            for (int w = 0; w < kTKW; ++w) zr[w] = w < kw ? zb[w * kTile + lane] : 0u;
            for (int r = wave; r < m; r += kTW) {
                const uint32_t *ar = g.a_packed + (size_t)r * kw;
                uint32_t par = ib[(r >> 5) * kTile + lane] >> (r & 31);
#pragma unroll
                for (int w = 0; w < kTKW; ++w)
                    if (w < kw) par += __builtin_popcount(ar[w] & zr[w]);
                acc |= par & 1u;
            }
        }
        if (acc) atomicOr((uint32_t *)bad + lane, 1u);
        __syncthreads();

        if (wave == 0) {  // per-lane exits and counters (vn_kernel's stream variant)
            unsigned long long v[7] = {0, 0, 0, 0, 0, 0, 0};
            bool fin = false;
            if (c.live) {
                const int it = itl[lane];
                const bool ok = bad[lane] == 0;  // Result.OK at this iteration (:231-241)
                fin = ok || it == max_iter - 1;  // else DATA_TRANSFER_NOT_OK (:244-253)
                if (fin) {
                    int err = 0;
                    if (!ok)  // main.py:130-138: u vs z^1 of a failed frame
                        for (int w = 0; w < kw; ++w) err += __builtin_popcount(Ut[w * kTile] ^ zb[w * kTile + lane]);
                    v[0] = 1;
                    v[1] = ok ? 0 : 1;
                    v[2] = (unsigned long long)err;
                    v[3] = ok ? (unsigned long long)it : 0;
                    v[4] = ok ? 1 : 0;
                    v[5] = nllr ? (unsigned long long)cntl[lane] : 0;
                    v[6] = (unsigned long long)(it + 1);
                    livel[lane] = 0;
                    want = true;
                } else {
                    itl[lane] = it + 1;
                }
                freshl[lane] = 0;
            }
            if (__ballot(fin) != 0ull) {
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const unsigned long long s = wave_sum(v[i]);
                    if (lane == 0 && s) atomicAdd(&ctr[i], s);
                }
            }
            bad[lane] = 0;
            cntl[lane] = 0;
        }
        for (int i = threadIdx.x; i < mw * kTile; i += blockDim.x) ib[i] = 0u;
        // zb is reused as the u-bit stage and cleared at the top of the loop
    }
    count_rare_rows(st, c.tseq, kTW);
}

}  // namespace

size_t tile64_lds_bytes(const DevGraph &g) {
    if (!g.std_form || !g.a_packed || g.k <= 0 || g.k > 32 * kTKW || g.max_row_deg > kTW * kTK) return 0;
    const size_t b = tile_layout(g.k, g.m).total;
    return b <= kTileLdsMax ? b : 0;
}

// The long codes: the 16-frame sub-tile decoder (tile_sub.hip) for
// wimax_2304_0.5, the north-star code; the 8-frame decoder (tile8.hip) for
// the r3/4 codes, whose column sums of 16 frames do not fit in LDS (their
// graphs keep E in 8-frame blocks, DevGraph::ef = 8).
static bool sub_enabled(const DevGraph &g) { return g.ef == kTile && sub_frames(g) == 16; }

size_t tile_lds_bytes(const DevGraph &g) {
    const size_t b = tile64_lds_bytes(g);
    if (b) return b;
    if (g.ef == 8) return tile8_lds_bytes(g);
    return sub_enabled(g) ? sub_lds_bytes(g) : 0;
}

const char *tile_kernel_name(const DevGraph &g) {
    if (tile64_lds_bytes(g)) return "tile_kernel";
    if (g.ef == 8) return tile8_lds_bytes(g) ? (g.t8pair ? "tile8_kernel:pair" : "tile8_kernel") : "";
    if (sub_enabled(g) && sub_lds_bytes(g)) return "tile_sub_kernel";
    return "";
}

// LDPC_TILE=0 forces the separate CN/VN launches (A/B, tests)
bool use_tile(const DevGraph &g) {
    static const int force = [] {
        const char *e = getenv("LDPC_TILE");
        return e ? atoi(e) : -1;
    }();
    return force != 0 && tile_lds_bytes(g) > 0;
}

// Streaming Monte-Carlo in one persistent launch per SNR point: tile_stream_kernel
// (64 frames per workgroup), tile_sub_stream_kernel (16-frame sub-tiles,
// wimax_2304_0.5) or tile8_stream_kernel (8-frame sub-tiles: the r3/4 codes).  LDPC_TILE_STREAM=0 falls back to the separate launches.
static bool sub16(const DevGraph &g) { return sub_enabled(g) && sub_frames(g) == 16; }
bool use_tile_stream(const DevGraph &g) {
    const char *e = getenv("LDPC_TILE_STREAM");
    if (e && atoi(e) == 0) return false;
    const size_t lds = tile64_lds_bytes(g);
    // + the kernel's static per-lane state (itl, freshl: 2 x 64 ints; gidx: 64
    // frame indices; the refill flag)
    if (lds) return lds + 2 * kTile * sizeof(int) + kTile * sizeof(long long) + 16 <= kTileLdsMax;
    if (g.ef == 8) {  // tile8.hip: tile8_stream_kernel (LDPC_TILE8_STREAM=0: the split streaming loop)
        const char *e8 = getenv("LDPC_TILE8_STREAM");
        return !(e8 && atoi(e8) == 0) && tile8_stream_lds_bytes(g) > 0;
    }
    return sub16(g);
}

hipError_t launch_tile_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                              int snr_point, double sigma, int64_t frame0, int64_t total, unsigned long long *next,
                              unsigned long long *ctr, int64_t handoff, hipStream_t s) {
    const size_t lds = tile64_lds_bytes(g);
    if (!lds && g.ef == 8)
        return launch_tile8_stream(g, st, max_iter, nllr, seed, snr_point, sigma, frame0, total, next, ctr, handoff,
                                   s);
    if (!lds && sub16(g))
        return launch_tile_sub_stream(g, st, max_iter, nllr, seed, snr_point, sigma, frame0, total, next, ctr,
                                      handoff, s);
    if (!lds || !g.a_packed || !st.ubits || 2 * st.ntiles > st.nslots) return hipErrorInvalidValue;
    tile_stream_kernel<<<st.ntiles, 64 * kTW, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx, g.row_ptr,
                                                        kAtanhCoef, seed, snr_point, sigma, frame0, total, next, ctr);
    return hipGetLastError();
}

hipError_t launch_tile(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s) {
    if (2 * st.ntiles > st.nslots) return hipErrorInvalidValue;  // two rare-row buffers per tile
    const size_t lds = tile64_lds_bytes(g);
    if (!lds && g.ef == 8) return launch_tile8(g, st, max_iter, nllr, s);
    if (!lds) return sub_enabled(g) ? launch_tile_sub(g, st, max_iter, nllr, s) : hipErrorInvalidValue;
    tile_kernel<<<st.ntiles, 64 * kTW, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx, g.row_ptr);
    return hipGetLastError();
}

}  // namespace ldpc
