// tile_sub.hip -- the tile-resident parity decoder for long codes (gfx950).
//
// tile_kernels.hip decodes 64 frames per workgroup with the column sums
// S_j = ((0 + E_r0j) + E_r1j) + ... (rows ascending: scipy csr_matvec of E^T,
// the reference's rounding order, python_ldpc_app/spa_decoder.py:173-185)
// kept in LDS: k x 64 x 8 B, which holds only for k <= ~300.  The WiMAX 2304
// codes (k = 1152, 1728) fit when a workgroup decodes a SUB-tile of F = 16 or
// 8 frames (S = k x F x 8 B: 147 KB / 110 KB).  A wavefront instruction then
// covers Q = 64/F edges of F frames: lane = j*F + f (lane group j, frame f).
//
// Row r's edges are split into 16 contiguous wavefront chunks as in
// tile_kernel (wavefront w: positions [w*C, w*C + C), C = ceil(deg/16)), and a
// chunk into Q contiguous lane-group pieces of CS = ceil(C/Q) edges: lane group
// j holds positions j*CS .. j*CS + CS - 1 of the chunk in register slots
// 0..CS-1.  The left-to-right product P = t0 * t1 * ... (:151-152) crosses lane
// groups inside the wavefront: starting from the prefix P of the wavefront
// before it, every lane multiplies its own slots in order; lane group j's
// result is the prefix through group j, moved to group j+1 (permlane swaps;
// ds_bpermute for Q = 8)
// before group j+1's turn.  Groups with no edges are skipped.  Each wavefront
// runs the hop-first pipeline
//
//   body(r):  hop(r)   this wavefront's piece of row r's product;
//             P3(r-1)  E_new = 2 atanh(clip(P/t)) (:159-168), stored, added
//                      into S (LDS, per lane: column of its edge, its frame)
//                      after the overlapping wavefronts' P3(r-2) (sub_p3);
//             P1(r+1)  L[col], E_old, t = tanh((L - E_old)/2) (:138-146,
//                      :260-268).
//
// The default decoder of wimax_2304_0.5 (F = 16, Q = 4: the product crosses
// lane groups with v_permlane16/32_swap); bit-identical to the split path.
// (An F = 8 form of this kernel for the r3/4 codes was retired in round 3:
// tile8.hip decodes them, with E in 8-frame blocks.)
//
// Per edge and iteration the HBM traffic is the algorithmic 16 B (E_old read,
// E_new write) plus the L[col] gather (8 B, L2/MALL): the split CN/VN
// launches this replaces move 24 + 8 B plus the gathers.  The identity column
// k+r of a [A | I] graph has row r's last edge only; its posterior
// ch + (0 + E) is final when row r is.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "cn_common.h"
#include "frame_source.h"
#include "spa_device.h"
#include "spa_math.h"
#include "tile_common.h"

namespace ldpc {
namespace {

// wavefronts per workgroup: kSubWaves (16, spa_device.h; 12 wavefronts with
// 168 registers each spilled less but measured 6 % slower, profiles/r4z_ab)
constexpr int kSW = kSubWaves;
// -DLDPC_SUB_TIMERS: diagnostic build (never the product) -- s_memtime phase
// timers per wavefront, printed for two workgroups at the end of the launch:
// hop wait, hop, P3 chain wait, P3 math + stores, P3 order wait, P3 adds, P1
#ifdef LDPC_SUB_TIMERS
#define SUB_NT 7
#define SUB_STAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SUB_ADD(c, i, a, b) ((c).tm[i] += (b) - (a))
#else
#define SUB_STAMP(v)
#define SUB_ADD(c, i, a, b)
#endif
constexpr size_t kSubLdsMax = 163840;


template <int Q>
struct SubCfg {
    static constexpr int F = kTile / Q;           // frames per workgroup
    static constexpr int K = Q == 4 ? 10 : 8;  // slots per lane: row degree <= kSW * Q * K
};

// The product crosses lane groups by v_permlane16/32_swap (Q = 4) or
// ds_bpermute (Q = 8); the wavefront carrying the chain runs at raised issue
// priority; the message stream E (read once, written once per pass) is
// non-temporal, as in tile_kernels.hip.  Pipeline: body(r) = hop(r), P3(r-1),
// P1(r+1) -- the chain of row r runs while the other wavefronts are still in
// P3(r-1); the S additions of a row wait on the per-row P3 completion counts,
// and the chain slots are reused every 4 rows.
constexpr int kSR = 4;  // chain slots
// P1 loads and evaluates tanh for all K slots of a lane, branch-free: slots
// past the chunk's CS hold clamped, valid data (their t ends as 1.0 and is never
// used), and the straight-line code lets each slot's math wait only for its own
// loads (+2.7 % over a per-slot branch, profiles r2x logs); the hop multiplies
// all K slots of every lane group (the padded 1.0s are exact no-ops).  P3
// reads clamped column indices for every slot and adds each slot's E_new into
// its column sum with one ds_add_f64 (slots past the piece add into `dummy`):
// the same IEEE add of the same operands as read / add / write, rows ordered
// by the p3dep waits; ds_add_f64 rounds to nearest even and, unlike the other
// LDS float atomics, never flushes denormals (LLVM SIISelLowering emits it for
// workgroup-scope fadd only on that basis; +2 %, profiles/r4za_ab).  A fresh
// streaming frame's lanes (and iteration 0) read no E_old: M = L - 0.0 == L.
// Measured and not kept (profiles/ READMEs; git history has the code): tanh
// groups of 2-3 slots in lockstep (spills), guarded per-slot P1/P3 forms,
// skipping the padded slot K-1 (0.4375), sc1 E_new stores (0.436), uint16
// index staging (0.417), 12 wavefronts per workgroup (0.426).
// Logical wavefront (chunk position in a row) of hardware wavefront hw: the
// four wavefronts of one SIMD (hw = s, s+4, s+8, s+12) take four consecutive
// chunk positions, so each SIMD holds one contiguous quarter of every row's
// chain and its P3 neighbours.  +1.3 % over the identity map, static and
// streaming (profiles/r2at_wave_map; pairs of positions per SIMD measured the
// same, spin waits at a lower issue priority +0.2 %).
__device__ __forceinline__ int sub_wave(int hw) { return (hw & 3) * (kSW / 4) + (hw >> 2); }
// E_new stores through a buffer resource: a slot past the lane's piece (or a
// frame-less lane) stores at kSubOOB, past num_records, which the hardware
// drops -- no branch per slot, so every memory operation of the row loop is
// unconditional and the compiler's vmcnt waits count exactly (with branches
// it waited for this row's stores before P1's first request)
typedef unsigned int sub_u2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kSubOOB = 0xfffffff0u;
__device__ __forceinline__ void st_sub_msg(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(sub_u2, v), r, off, 0, 2 /* nt */);
}
// E_old loads the same way: at kSubOOB (iteration 0, a fresh frame) the
// hardware returns 0 without a memory request
__device__ __forceinline__ double ld_sub_msg(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 2 /* nt */));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sub_rsrc(const void *base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)min(bytes, (size_t)0x7fffffff),
                                            0x00020000);
}

// Column indices of the rows in flight, staged per wavefront in LDS as 16-bit
// values one row ahead of their P1 (a ring of 3 rows: P3(r-1), P1(r+1) and the
// staging of row r+2 in body(r)), so neither P1's posterior gather nor P3 waits
// on an index load from L2.
constexpr int kCRing = 3;
struct SubLayout {
    size_t S, math, slot, zb, ib, lane_i, flags, dummy, cidx, total;
};
__host__ __device__ constexpr int sub_k(int F) { return F == 16 ? SubCfg<4>::K : 0; }
__host__ __device__ inline SubLayout sub_layout(int k, int m, int F) {
    SubLayout t;
    size_t o = 0;
    t.S = o;  // [k][F] column sums
    o = al16(o + (size_t)k * F * sizeof(double));
    t.math = o;
    o = al16(o + sizeof(MathLds));
    t.slot = o;  // [kSR][F] chain slots
    o = al16(o + kSR * (size_t)F * sizeof(double));
    t.zb = o;  // [kw][F] z^1 bits of the A columns
    o = al16(o + (size_t)((k + 31) / 32) * F * sizeof(uint32_t));
    t.ib = o;  // [mw][F] z^1 bits of the identity columns (adjacent to zb)
    o = al16(o + (size_t)((m + 31) / 32) * F * sizeof(uint32_t));
    t.lane_i = o;  // bad[F], nllr count[F], live[F]
    o = al16(o + 3 * (size_t)F * sizeof(int));
    t.flags = o;  // chain flag[kSR], tiny[kSR], tiny sequence, running, P3 rows done[kSW]
    o = al16(o + (2 * kSR + 2 + kSW) * sizeof(int));
    t.dummy = o;  // [F] target of the identity lane's masked-off S update
    o = al16(o + (size_t)F * sizeof(double));
    t.cidx = o;  // [kCRing][kSW][64/F * K] uint16 column indices (one wavefront chunk per row)
    o = al16(o + (size_t)kCRing * kSW * (64 / F) * sub_k(F) * sizeof(uint16_t));
    t.total = o;
    return t;
}

struct SubChunk {
    int deg, c0, cnt, CS;
};
__device__ __forceinline__ SubChunk sub_chunk(const int *__restrict__ row_ptr, int r, int wave, int Q) {
    SubChunk c;
    const int beg = row_ptr[r];
    c.deg = row_ptr[r + 1] - beg;
    const int C = (c.deg + kSW - 1) / kSW;
    c.c0 = beg + wave * C;
    c.cnt = max(0, min(c.deg - wave * C, C));
    c.CS = (C + Q - 1) / Q;
    return c;
}

template <int Q>
struct SubCtx {
    static constexpr int F = SubCfg<Q>::F;
    static constexpr int K = SubCfg<Q>::K;
    const int *__restrict__ col_idx;
    const int *__restrict__ row_ptr;
    // per-lane bases: element (item) of this lane's frame at [item * 64]
    double *Eb;
    double *Lb;
    const double *Cb;
    double *Tb;     // rare-row scratch of this workgroup, element (pos) at [pos * F]; two buffers
    size_t tbuf;    // doubles between them (rare rows alternate: tile_kernels.hip)
    double *S;      // LDS, element (col) at [col * F]
    double *dummy;  // LDS, this lane's frame
    double *slot;   // LDS, chain slot s at [s * F]
    uint32_t *ib;   // LDS, word w at [w * F]
    uint16_t *cidx; // LDS, this wavefront's index ring: row slot s, position p at [s * kSW * Q * K + p]
    int m;
    int *flag, *tinyf, *tseq, *p3row;
    const int *p3dep;
    LdsTanh ttab;
    LdsAtanh ltab;
    AtanhCoef ac;   // kernel-argument coefficients (when coef_arg)
    bool coef_arg;  // P3 uses ac instead of coef_load() (compile-time per kernel)
    // uniform (SGPR) tile bases + this lane's byte offset: every access is a
    // 32-bit per-lane offset from a scalar base (global_load ... v_off, s_base)
    const char *Eu, *Lu, *Cu;
    __amdgpu_buffer_rsrc_t rE;  // the tile's E for masked stores without a branch (sub_p3_body)
    uint32_t lo8;
    int k, wave, j, f;
    int ep0;
    bool first, live;
    bool fresh;  // streaming: this lane's frame is on its first pass (M = L - 0, L = ch)
    int ntiny;
#ifdef LDPC_SUB_TIMERS
    mutable uint64_t tm[SUB_NT];
#endif
};

// this lane's edge count in chunk rc, and the edge of its slot i (clamped
// into the chunk: slots past the piece load the chunk's last edge again)
template <int Q>
__device__ __forceinline__ int sub_nj(const SubCtx<Q> &c, const SubChunk &rc) {
    return max(0, min(rc.cnt - c.j * rc.CS, rc.CS));
}
template <int Q>
__device__ __forceinline__ int sub_edge(const SubCtx<Q> &c, const SubChunk &rc, int i) {
    return rc.c0 + min(c.j * rc.CS + i, rc.cnt - 1);
}
// element (item, this lane's frame) of a tile array: item * 64 * 8 + lane * 8 bytes
template <int Q>
__device__ __forceinline__ uint32_t sub_off(const SubCtx<Q> &c, int item) {
    return ((uint32_t)item << 9) + c.lo8;
}
template <int Q>
__device__ __forceinline__ double *sub_l(const SubCtx<Q> &c, int col) {
    return (double *)(c.Lu + sub_off(c, col));
}
template <int Q>
__device__ __forceinline__ const double *sub_c(const SubCtx<Q> &c, int col) {
    return (const double *)(c.Cu + sub_off(c, col));
}
template <int Q>
__device__ __forceinline__ int sub_col(const SubCtx<Q> &c, int edge) {
    return *(const int *)((const char *)c.col_idx + ((uint32_t)edge << 2));
}
// This lane's piece of row r's staged column indices: slot i at [i].  The
// staging wrote every position < Q*K (past the chunk: the clamped last
// column), and j*CS + i < Q*K for every slot, so no clamp is needed here and
// each slot's read is an immediate offset from one address per row.
template <int Q>
__device__ __forceinline__ const uint16_t *sub_lcols(const SubCtx<Q> &c, int r, const SubChunk &rc) {
    return c.cidx + (r % kCRing) * kSW * Q * SubCfg<Q>::K + c.j * rc.CS;
}
// Byte offset of this lane's slot 0 of chunk rc in the tile's E; slot i is at
// + i * 512.  Slots past the lane's piece are NOT clamped: their loads read
// other edges (past the tile's last edge: the buffer returns 0) and their
// values are discarded (t = 1.0, the store dropped at kSubOOB).
template <int Q>
__device__ __forceinline__ uint32_t sub_eoff(const SubCtx<Q> &c, const SubChunk &rc) {
    return ((uint32_t)(rc.c0 + c.j * rc.CS) << 9) + c.lo8;
}
// Staging of row q's indices into the ring: issue (one index per lane, lanes <
// the chunk size) early, commit to LDS once the wavefront has waited on its
// other loads anyway.
template <int Q>
__device__ __forceinline__ int sub_stage_issue(const SubCtx<Q> &c, int q) {
    // always one load (an in-range edge): a conditional load into a register
    // also written with 0 makes the compiler wait for every outstanding
    // memory operation (this row's E_new stores) before P1's first request
    const SubChunk rc = sub_chunk(c.row_ptr, min(q, c.m - 1), c.wave, Q);
    const int L = threadIdx.x & 63;
    return sub_col(c, min(max(rc.c0 + min(L, rc.cnt - 1), 0), c.row_ptr[c.m] - 1));
}
template <int Q>
__device__ __forceinline__ void sub_stage_commit(const SubCtx<Q> &c, int q, int v) {
    if (q >= c.m) return;
    constexpr int W = Q * SubCfg<Q>::K;  // positions per wavefront chunk (40 / 64)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if ((int)(threadIdx.x & 63) < W) c.cidx[(q % kCRing) * kSW * W + (threadIdx.x & 63)] = (uint16_t)v;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// P1: t = tanh((L[col] - E_old)/2) for this lane's slots; returns whether
// some lane's own edge has |t| <= 1e-10 (:159).  E_old is requested first
// (independent of the column indices), then the indices, then the posterior
// gather that needs them.
template <int Q>
__device__ __forceinline__ bool sub_p1(const SubCtx<Q> &c, int r, const SubChunk &rc, double (&t)[SubCfg<Q>::K]) {
    constexpr int K = SubCfg<Q>::K;
    bool tiny = false;
    const int sv = sub_stage_issue(c, r + 1);  // row r+1's indices, committed below
    if (rc.cnt > 0) {
        const int nj = sub_nj(c, rc);
        const int njt = c.live ? nj : 0;  // the |t| <= 1e-10 vote: frame-less lanes abstain
        const uint16_t *lc = sub_lcols(c, r, rc);
        const uint32_t eoff = sub_eoff(c, rc);
        // iteration 0 / a fresh streaming frame: M = L
        const bool noE = c.first || c.fresh;
        int col[K];
        double eo[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            // iteration 0 and a fresh frame's lanes read no E_old (on a
            // streaming pass most slots hold fresh frames)
            eo[i] = ld_sub_msg(c.rE, noE ? kSubOOB : eoff + (uint32_t)i * (kTile * sizeof(double)));
            col[i] = lc[i];
        }
        const char *Lsrc = c.first ? c.Cu : c.Lu;  // iteration 0: M = ch (:85-90); uniform
#pragma unroll
        for (int i = 0; i < K; ++i) t[i] = ld_l2((const double *)(Lsrc + sub_off(c, col[i])));
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const double M = noE ? t[i] : t[i] - eo[i];  // :85-90 / :260-268
            const double d = M * 0.5;
            // :138-146 as np_tanh of M/2 clamped to +-17.5 (spa_math.h
            // tanh_half_clipped: equal to the reference's clip for every M)
            double th[1] = {dfrom(dbits(fmin(fabs(d), 17.5)) | (dbits(d) & 0x8000000000000000ull))};
            np_tanh_n<1, LdsTanh, true>(th, c.ttab);
            const double tv = th[0];
            tiny |= i < njt && !(fabs(tv) > kTiny);
            // slots past this lane's piece: 1.0, an exact no-op in the chain product
            t[i] = i < nj ? tv : 1.0;
        }
    }
    sub_stage_commit(c, r + 1, sv);
    return __ballot(tiny) != 0ull;
}

// Lane-group hand-over for Q = 4 (lane = j*16 + f: group j is DPP row j) with
// gfx950's v_permlane16_swap / v_permlane32_swap (VALU, no LDS round trip):
// permlane16_swap(x, x) -> {[x0 x0 x2 x2], [x1 x1 x3 x3]} (rows),
// permlane32_swap(x, x) -> {[x0 x1 x0 x1], [x2 x3 x2 x3]}.
__device__ __forceinline__ uint32_t p16(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t p32(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
// value of group jj moved into group jj+1 (other groups: don't care)
__device__ __forceinline__ double group_up4(double v, int jj) {
    const uint64_t u = dbits(v);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    if (jj == 1) {  // row 1 -> row 2: [x0 x1 x0 x1] then its odd rows
        lo = p16(p32(lo, 0), 1);
        hi = p16(p32(hi, 0), 1);
    } else {  // row 0 -> 1, row 2 -> 3
        lo = p16(lo, 0);
        hi = p16(hi, 0);
    }
    return dfrom(((uint64_t)hi << 32) | lo);
}


// P * t[0] * ... * t[n-1] as exactly n dependent multiplies (a uniform branch
// on n selects a straight-line sequence; slots past a lane's piece hold 1.0)
template <int K, int N>
struct SubMul {
    static __device__ __forceinline__ double run(double P, const double (&t)[K], int n) {
        if (n == N) {
#pragma unroll
            for (int i = 0; i < N; ++i) P = P * t[i];
            return P;
        }
        return SubMul<K, N - 1>::run(P, t, n);
    }
};
template <int K>
struct SubMul<K, 0> {
    static __device__ __forceinline__ double run(double P, const double (&)[K], int) { return P; }
};

// hop: this wavefront's chunk of row r's left-to-right product.  Round jj
// multiplies lane group jj's slots into the running product (every lane
// computes; group jj's lanes hold the value that matters) and moves it to
// group jj+1.
template <int Q>
__device__ __forceinline__ void sub_hop(const SubCtx<Q> &c, int r, const double (&t)[SubCfg<Q>::K], bool tiny) {
    constexpr int F = SubCfg<Q>::F, K = SubCfg<Q>::K;
    const SubChunk rc = sub_chunk(c.row_ptr, r, c.wave, Q);
    if (rc.deg == 0) return;  // spa_decoder.py:115-122
    const int s = r & (kSR - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    double *sl = c.slot + s * F;
    double P = 1.0;  // 1.0 * t0 == t0 exactly
    SUB_STAMP(h0);
    if (c.wave != 0) {
        wait_flag<false>(c.flag + s, ep + c.wave);
        P = *sl;
    }
    SUB_STAMP(h1);
    SUB_ADD(c, 0, h0, h1);
    __builtin_amdgcn_s_setprio(2);
    int last = -1;
    if (Q == 4 && rc.cnt > 0) {
        // branch-free: every lane group multiplies all K slots (slots past its
        // piece and every slot of a group past the chunk hold 1.0, sub_p1:
        // exact no-ops), so the product ends in group 3 -- no uniform
        // branches between the dependent multiplies
#pragma unroll
        for (int jj = 0; jj < Q; ++jj) {
#pragma unroll
            for (int i = 0; i < K; ++i) P = P * t[i];
            if (jj + 1 < Q) P = group_up4(P, jj);
        }
        last = Q - 1;
    } else {
#pragma unroll
        for (int jj = 0; jj < Q; ++jj) {
            if (jj * rc.CS < rc.cnt) {  // lane group jj holds edges of this chunk (uniform)
                const double Pl = SubMul<K, K>::run(P, t, rc.CS);
                last = jj;
                if (jj + 1 < Q && (jj + 1) * rc.CS < rc.cnt)
                    P = group_up4(Pl, jj);
                else
                    P = Pl;
            }
        }
    }
    if ((threadIdx.x & 63) == 0) {
        if (c.wave == 0)
            lds_st(c.tinyf + s, tiny ? 1 : 0);
        else if (tiny)
            lds_st(c.tinyf + s, 1);
    }
    if (c.j == last) *sl = P;
    lds_release();
    if ((threadIdx.x & 63) == 0) lds_st(c.flag + s, ep + c.wave + 1);
    __builtin_amdgcn_s_setprio(0);
    SUB_STAMP(h2);
    SUB_ADD(c, 1, h1, h2);
}

// P3: E_new of this lane's slots of row r, stored and folded into S; the
// identity column's posterior and z^1 bit.
// row r-1's P3 by the wavefronts whose column spans overlap this one's (sub_p3)
template <int Q>
__device__ __forceinline__ void sub_order(const SubCtx<Q> &c, int r) {
    if (r > 0) {
        const int d = ld_table(c.p3dep, r * kSW + c.wave);
        for (int v = d & 0xff; v <= (d >> 8); ++v) wait_ge<false>(c.p3row + v, r);
    }
}
template <int Q>
__device__ __forceinline__ void sub_p3_body(SubCtx<Q> &c, int r, double (&t)[SubCfg<Q>::K]) {
    constexpr int F = SubCfg<Q>::F, K = SubCfg<Q>::K;
    const SubChunk rc = sub_chunk(c.row_ptr, r, c.wave, Q);
    if (rc.deg == 0) return;
    const int s = r & (kSR - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    // the identity column k + r is the row's last edge (an [A | I] graph):
    // the lane whose piece ends there requests its channel LLR now, ahead of
    // the chain wait (+1 % with the late S-order wait below, profiles/r5n_ab)
    // (every lane requests it: a conditional load leaves the compiler's
    // vmcnt count inexact; the 16 frames' 128 B are one line for all lanes)
    const double chI = *sub_c(c, c.k + r);
    SUB_STAMP(q0);
    wait_flag<false>(c.flag + s, ep + kSW);
    SUB_STAMP(q1);
    SUB_ADD(c, 2, q0, q1);
    const bool tiny_row = uniform(lds_ld(c.tinyf + s)) != 0;
    if (rc.cnt == 0) {  // no edges here (short rows): still take part in a rare row's parking count
        sub_order(c, r);
        if (tiny_row) {
            c.ntiny += 1;
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_fetch_add(c.tseq, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            wait_flag<false>(c.tseq, c.ntiny * kSW);
        }
        return;
    }
    const double P = c.slot[s * F];
    const int nj = sub_nj(c, rc);
    const uint16_t *lc = sub_lcols(c, r, rc);
    int col[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        col[i] = lc[i];  // clamped copy past the chunk: a valid column
    if (!tiny_row) {
        // q = P/t (div_nr: the IEEE quotient without the scaling steps,
        // cn_common.h), then E_new = 2 atanh(clip(q)) (:159-168) -- or 2q when
        // every quotient of the wavefront is below 2^-27, where that is exact
        // (spa_math.h kAtanhIdent; the common case on long rows at low SNR)
        bool big = false;
        const double lim = c.live ? kAtanhIdent : INFINITY;  // frame-less lanes do not vote
        if (div_nr_ok(c.live ? P : 1.0)) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < rc.CS) {
                    t[i] = div_nr(P, t[i]);
                    big |= !(fabs(t[i]) < lim);
                }
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < rc.CS) {
                    t[i] = P / t[i];
                    big |= !(fabs(t[i]) < lim);
                }
        }
        if (__ballot(big) == 0ull) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < rc.CS) t[i] = 2.0 * t[i];
        } else {
            const AtanhCoef ac = c.coef_arg ? c.ac : coef_load();  // scalar loads here (cn_common.h)
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < rc.CS) t[i] = 2.0 * atanh_f(clip_cl(t[i]), c.ltab, ac);
        }
    } else {
        // rare: q = in-order product of the others (np.prod(np.delete(...)),
        // :164) for an edge with |t| <= 1e-10; t parked at row positions
        const int rb = c.row_ptr[r];
        double *tb = c.Tb + (c.ntiny & 1) * c.tbuf;  // the next rare row parks in the other buffer
#pragma unroll
        for (int i = 0; i < K; ++i)
            if (i < rc.CS && i < nj) tb[(size_t)(sub_edge(c, rc, i) - rb) * F] = t[i];
        __builtin_amdgcn_s_waitcnt(0);  // scratch stores have reached L2
        c.ntiny += 1;
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c.tseq, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_flag<false>(c.tseq, c.ntiny * kSW);
        const AtanhCoef ac = c.coef_arg ? c.ac : coef_load();  // scalar loads here (cn_common.h)
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if (i < rc.CS) {
                const double ti = t[i];
                double q;
                if (fabs(ti) > kTiny || i >= nj) {
                    q = P / ti;
                } else {
                    const int pos = sub_edge(c, rc, i) - rb;
                    q = 1.0;
                    bool fst = true;
                    for (int p = 0; p < rc.deg; ++p) {
                        if (p == pos) continue;
                        const double t2 = ld_l2(tb + (size_t)p * F);
                        q = fst ? t2 : q * t2;
                        fst = false;
                    }
                }
                t[i] = 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
            }
        }
    }
    {
        const uint32_t eoff = sub_eoff(c, rc);
#pragma unroll
        for (int i = 0; i < K; ++i)  // nj <= CS
            st_sub_msg(c.rE, (i < nj && c.live) ? eoff + (uint32_t)i * (kTile * sizeof(double)) : kSubOOB, t[i]);
    }
    // S_col += E_new, rows ascending (a column occurs once per row: no two
    // lanes of a row share (col, frame)); the identity edge goes to `dummy`
    double EnI = 0.0;
    int colI = -1;
    double *sp[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const bool own = i < nj;  // nj <= CS
        const bool a = own && col[i] < c.k;
        sp[i] = a ? c.S + (size_t)col[i] * F : c.dummy;
        if (own && !a) {
            EnI = t[i];
            colI = col[i];
        }
    }
    // S order: only the additions wait for the overlapping wavefronts' row
    // r-1 (the math and the E_new stores above run meanwhile)
    SUB_STAMP(q2);
    SUB_ADD(c, 3, q1, q2);
    sub_order(c, r);
    SUB_STAMP(q3);
    SUB_ADD(c, 4, q2, q3);
#pragma unroll
    for (int i = 0; i < K; ++i)  // one ds_add_f64 per slot; slots past the piece add into `dummy` (never read)
        __hip_atomic_fetch_add(sp[i], t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (colI >= 0) {  // identity column: L = ch + (0 + E) (:173-185)
        const double Lj = chI + (0.0 + EnI);
        if (c.live) *sub_l(c, colI) = Lj;
        if (!(Lj < 0.0)) {
            const int q = colI - c.k;
            atomicOr(c.ib + (q >> 5) * F, 1u << (q & 31));
        }
    }
    SUB_STAMP(q4);
    SUB_ADD(c, 5, q3, q4);
}

// P3 of row r.  S_col must take its additions rows ascending.  Wavefront w's
// chunk of row r spans columns [first, last]; extended to the gap before it,
// the chunks of a row partition the columns, so waiting for row r-1's P3 by
// exactly the wavefronts whose extended spans overlap w's (g.p3dep, built on
// the host: ldpc_api.cpp sub_p3_deps) orders every column's additions by
// induction over the rows -- the neighbours, not all 16 wavefronts (the full
// row barrier this replaces cost early wavefronts up to 39 % of their time,
// profiles/r2an_phase_timers).  p3row[v] = 1 + the last row r of THIS pass
// whose P3 wavefront v finished; sub_p3_reset zeroes it between passes (after
// the barrier that ends a pass's rows), so the count never exceeds m + 1 however
// many passes a streaming launch makes.
template <int Q>
__device__ __forceinline__ void sub_p3(SubCtx<Q> &c, int r, double (&t)[SubCfg<Q>::K]) {
    sub_p3_body<Q>(c, r, t);
    lds_release();  // this row's S additions before the count
    if ((threadIdx.x & 63) == 0)
        lds_st(c.p3row + c.wave, r + 1);
}
// Between passes: every wavefront has finished (and waited on) the pass's
// P3s -- call after the barrier that ends the row loop, before the next one.
__device__ __forceinline__ void sub_p3_reset(int *p3row) {
    if (threadIdx.x < kSW) p3row[threadIdx.x] = 0;
}
// Chain-flag epoch of a pass: (pass * m) mod 2^26, so ep0 + r (masked again
// where used) neither overflows nor breaks the sequence of epochs across passes.
__device__ __forceinline__ int sub_epoch0(int pass, int m) {
    return (int)(((uint32_t)pass * (uint32_t)m) & 0x3ffffffu);
}

template <int Q>
__device__ __forceinline__ void sub_body(SubCtx<Q> &c, int r, int m, double (&tcur)[SubCfg<Q>::K], bool ycur,
                                         double (&toth)[SubCfg<Q>::K], bool &yoth) {
    if (r < m) sub_hop(c, r, tcur, ycur);
    if (r >= 1) sub_p3<Q>(c, r - 1, toth);
    SUB_STAMP(p0);
    if (r + 1 < m) yoth = sub_p1<Q>(c, r + 1, sub_chunk(c.row_ptr, r + 1, c.wave, Q), toth);
    SUB_STAMP(p1);
    SUB_ADD(c, 6, p0, p1);
}

template <int Q>
__global__ __launch_bounds__(64 * kSW, 1) void tile_sub_kernel(DevGraph g, DevState st, int max_iter, int nllr,
                                                               const int *__restrict__ col_idx,
                                                               const int *__restrict__ row_ptr, AtanhCoef ac) {
    constexpr int F = SubCfg<Q>::F, K = SubCfg<Q>::K;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const SubLayout ly = sub_layout(g.k, g.m, F);
    double *S = (double *)(lds + ly.S);
    MathLds &mlds = *(MathLds *)(lds + ly.math);
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + F;
    int *livel = cntl + F;
    int *flags = (int *)(lds + ly.flags);
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x / Q, sub = blockIdx.x % Q;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(mlds);
    for (int i = threadIdx.x; i < g.k * F; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * F; i += blockDim.x) zb[i] = 0u;
    for (int i = threadIdx.x; i < 2 * F; i += blockDim.x) bad[i] = 0;
    if (threadIdx.x < 2 * kSR) flags[threadIdx.x] = -1;
    if (threadIdx.x >= 2 * kSR && threadIdx.x < 2 * kSR + 2 + kSW) flags[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    const int wave = uniform(sub_wave(threadIdx.x >> 6));
    const int j = lane / F, f = lane % F;
    const int fr = tile * kTile + sub * F + f;  // this lane's frame
    if (wave == 0 && j == 0) livel[f] = st.done[fr] == 0 ? 1 : 0;
    __syncthreads();
    if (!st.tile_active[tile]) return;
    {  // a sub-tile with no live frame (a ragged batch's last tile) has nothing to do
        int any = 0;
#pragma unroll
        for (int ff = 0; ff < F; ++ff) any |= livel[ff];
        if (!any) return;  // block-uniform: LDS after the barrier
    }

    SubCtx<Q> c;
    c.col_idx = col_idx;
    c.row_ptr = row_ptr;
    const size_t lo = (size_t)sub * F + f;
    c.Eb = st.E + (size_t)tile * g.nnz * kTile + lo;
    c.Lb = st.L + (size_t)tile * g.n * kTile + lo;
    c.Cb = st.ch + (size_t)tile * g.n * kTile + lo;
    c.Eu = (const char *)(st.E + (size_t)tile * g.nnz * kTile);
    c.rE = sub_rsrc(c.Eu, (size_t)g.nnz * kTile * sizeof(double));
    c.Lu = (const char *)(st.L + (size_t)tile * g.n * kTile);
    c.Cu = (const char *)(st.ch + (size_t)tile * g.n * kTile);
    c.lo8 = (uint32_t)lo * 8u;
    c.Tb = st.T + (size_t)blockIdx.x * 2 * g.max_row_deg * F + f;
    c.tbuf = (size_t)g.max_row_deg * F;
    c.S = S + f;
    c.dummy = (double *)(lds + ly.dummy) + f;
    c.slot = (double *)(lds + ly.slot) + f;
    c.ib = ib + f;
    c.cidx = (uint16_t *)(lds + ly.cidx) + wave * Q * K;
    c.m = g.m;
    c.flag = flags;
    c.tinyf = flags + kSR;
    c.tseq = flags + 2 * kSR;
    c.p3row = flags + 2 * kSR + 2;
    c.p3dep = g.p3dep;
    c.ttab = LdsTanh{mlds.tanh};
    c.ltab = LdsAtanh{mlds.atanh};
    c.coef_arg = false;  // the static decoder loads them (1 dB: atanh on few rows)
    c.ac = ac;
    c.k = g.k;
    c.wave = wave;
    c.j = j;
    c.f = f;
    c.ntiny = 0;
    c.fresh = false;
#ifdef LDPC_SUB_TIMERS
    for (int i = 0; i < SUB_NT; ++i) c.tm[i] = 0;
#endif
    const int m = g.m;
    const int nthr = kSW * Q;       // (wavefront, lane group) pairs
    const int me = wave * Q + j;    // this lane's pair

    for (int it = 0; it < max_iter; ++it) {
        c.first = it == 0;
        c.live = livel[f] != 0;
        c.ep0 = sub_epoch0(it, m);
        double tA[K], tB[K];
        bool yA = false, yB = false;
        if (m > 0) {
            sub_stage_commit(c, 0, sub_stage_issue(c, 0));
            yA = sub_p1<Q>(c, 0, sub_chunk(row_ptr, 0, wave, Q), tA);
        }
        for (int r = 0; r <= m; r += 2) {
            sub_body<Q>(c, r, m, tA, yA, tB, yB);
            if (r + 1 <= m) sub_body<Q>(c, r + 1, m, tB, yB, tA, yA);
        }
        __syncthreads();  // every P3 done: S complete, identity bits set
        sub_p3_reset(c.p3row);

        // posteriors of the A columns (channel added after the sum), the
        // normalized-LLR count against the previous posterior (:210-228),
        // z^1 bits
        int my_cnt = 0;
        for (int col = me; col < g.k; col += nthr) {
            double *sp = c.S + (size_t)col * F;
            const double Sj = *sp;
            *sp = 0.0;
            const double chj = *sub_c(c, col);
            const double Lj = chj + Sj;
            if (nllr) {
                const double ap = c.first ? chj : ld_l2(sub_l(c, col));
                my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
            }
            if (c.live) *sub_l(c, col) = Lj;
            if (!(Lj < 0.0)) atomicOr(zb + (col >> 5) * F + f, 1u << (col & 31));
        }
        if (nllr && my_cnt) atomicAdd(cntl + f, my_cnt);
        __syncthreads();

        // syndrome (:191-204): parity of row r = popcount(A_r & (z^1)_A) +
        // (z^1)_{k+r}, A_r bit-packed
        uint32_t acc = 0u;
        for (int r = me; r < m; r += nthr) {
            const uint32_t *ar = g.a_packed + (size_t)r * kw;
            uint32_t par = ib[(r >> 5) * F + f] >> (r & 31);
            for (int w = 0; w < kw; ++w) par += __builtin_popcount(ar[w] & zb[w * F + f]);
            acc |= par & 1u;
        }
        if (acc) atomicOr((uint32_t *)bad + f, 1u);
        __syncthreads();

        if (wave == 0) {  // per-frame exits, as vn_kernel (static schedule)
            bool still = false;
            if (j == 0 && c.live) {
                if (nllr) {
                    const int cn = cntl[f];
                    st.nllr_cnt[fr] = cn;
                    if (st.nllr_hist)
                        st.nllr_hist[(size_t)fr * st.hist_stride + it] = g.k > 0 ? (double)cn / g.k : 0.0;
                }
                if (bad[f] == 0) {  // syndrome zero: Result.OK at this iteration (:231-241)
                    st.done[fr] = 1;
                    st.conv[fr] = it;
                    st.status[fr] = 0;
                    st.iters[fr] = it + 1;
                } else if (it == max_iter - 1) {  // Result.DATA_TRANSFER_NOT_OK (:244-253)
                    st.done[fr] = 1;
                    st.conv[fr] = -1;
                    st.status[fr] = 1;
                    st.iters[fr] = it + 1;
                } else {
                    still = true;
                }
            }
            const unsigned long long any = __ballot(still);
            if (j == 0) {
                livel[f] = still ? 1 : 0;
                bad[f] = 0;
                cntl[f] = 0;
            }
            if (lane == 0) flags[2 * kSR + 1] = any != 0ull ? 1 : 0;
        }
        for (int i = threadIdx.x; i < (kw + mw) * F; i += blockDim.x) zb[i] = 0u;
        __syncthreads();
        if (!flags[2 * kSR + 1]) break;
    }
    count_rare_rows(st, c.tseq, kSW);
#ifdef LDPC_SUB_TIMERS
    if ((blockIdx.x == 0 || blockIdx.x == 777) && (threadIdx.x & 63) == 0)
        printf("SUB b=%d w=%d hopw=%llu hop=%llu p3f=%llu p3m=%llu p3o=%llu p3s=%llu p1=%llu\n", (int)blockIdx.x,
               c.wave, (unsigned long long)c.tm[0], (unsigned long long)c.tm[1], (unsigned long long)c.tm[2],
               (unsigned long long)c.tm[3], (unsigned long long)c.tm[4], (unsigned long long)c.tm[5],
               (unsigned long long)c.tm[6]);
#endif
}

// Streaming Monte-Carlo on sub-tiles (tile_kernels.hip's tile_stream_kernel,
// at 16 frames per workgroup): every frame slot f is at its own iteration;
// after each pass a slot whose frame stopped adds that frame's counters
// (count_kernel's definitions, main.py:130-138) and takes the next frame
// index from one device counter; the frame is generated in place (gen_slots:
// ch and L = ch, so its next pass forms M = L - 0, its iteration 0).  Each
// frame decodes exactly as in the static schedule, so the counters are
// identical.  A workgroup exits once the supply is out and its slots drained.
template <int Q>
__global__ __launch_bounds__(64 * kSW, 1) void tile_sub_stream_kernel(
    DevGraph g, DevState st, int max_iter, int nllr, const int *__restrict__ col_idx,
    const int *__restrict__ row_ptr, AtanhCoef ac, uint64_t seed, int snr_point, double sigma, int64_t frame0,
    int64_t total, unsigned long long *next, unsigned long long *ctr, int64_t handoff) {
    constexpr int F = SubCfg<Q>::F, K = SubCfg<Q>::K;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int itl[F], freshl[F];
    __shared__ long long gidx[F];  // refill: slot f's new frame index (< 0: none)
    __shared__ int nref;           // refill: some slot took a frame this pass
    const SubLayout ly = sub_layout(g.k, g.m, F);
    double *S = (double *)(lds + ly.S);
    MathLds &mlds = *(MathLds *)(lds + ly.math);
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + F;
    int *livel = cntl + F;
    int *flags = (int *)(lds + ly.flags);
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x / Q, sub = blockIdx.x % Q;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(mlds);
    for (int i = threadIdx.x; i < g.k * F; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * F; i += blockDim.x) zb[i] = 0u;
    for (int i = threadIdx.x; i < 2 * F; i += blockDim.x) bad[i] = 0;
    if (threadIdx.x < 2 * kSR) flags[threadIdx.x] = -1;
    if (threadIdx.x >= 2 * kSR && threadIdx.x < 2 * kSR + 2 + kSW) flags[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    const int wave = uniform(sub_wave(threadIdx.x >> 6));
    const int j = lane / F, f = lane % F;
    const int lane64 = sub * F + f;
    const bool slot_lane = wave == 0 && j == 0;  // the lane that owns frame slot f
    bool want = slot_lane;
    if (slot_lane) {
        livel[f] = 0;
        itl[f] = 0;
        freshl[f] = 0;
    }

    SubCtx<Q> c;
    c.col_idx = col_idx;
    c.row_ptr = row_ptr;
    const size_t lo = (size_t)lane64;
    c.Eb = st.E + (size_t)tile * g.nnz * kTile + lo;
    c.Lb = st.L + (size_t)tile * g.n * kTile + lo;
    c.Cb = st.ch + (size_t)tile * g.n * kTile + lo;
    c.Eu = (const char *)(st.E + (size_t)tile * g.nnz * kTile);
    c.rE = sub_rsrc(c.Eu, (size_t)g.nnz * kTile * sizeof(double));
    c.Lu = (const char *)(st.L + (size_t)tile * g.n * kTile);
    c.Cu = (const char *)(st.ch + (size_t)tile * g.n * kTile);
    c.lo8 = (uint32_t)lo * 8u;
    c.Tb = st.T + (size_t)blockIdx.x * 2 * g.max_row_deg * F + f;
    c.tbuf = (size_t)g.max_row_deg * F;
    c.S = S + f;
    c.dummy = (double *)(lds + ly.dummy) + f;
    c.slot = (double *)(lds + ly.slot) + f;
    c.ib = ib + f;
    c.cidx = (uint16_t *)(lds + ly.cidx) + wave * Q * K;
    c.m = g.m;
    c.flag = flags;
    c.tinyf = flags + kSR;
    c.tseq = flags + 2 * kSR;
    c.p3row = flags + 2 * kSR + 2;
    c.p3dep = g.p3dep;
    c.ttab = LdsTanh{mlds.tanh};
    c.ltab = LdsAtanh{mlds.atanh};
    c.coef_arg = kStreamCoefArg;
    c.ac = ac;
    c.k = g.k;
    c.wave = wave;
    c.j = j;
    c.f = f;
    c.ntiny = 0;
    c.first = false;
    const int m = g.m;
    const int nthr = kSW * Q;
    const int me = wave * Q + j;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + lane64;

    for (int pass = 0;; ++pass) {
        if (wave == 0) {  // refill: slots without a frame take the next indices (generated below)
            // hand-off: once the supply is out and at most `handoff` frames
            // are still running anywhere, stop here and leave them to the
            // column-parallel tail (ldpc_api.cpp mc_stream_point): a running
            // frame costs this workgroup a full pass per iteration
            int stop = 0;
            if (handoff > 0 && lane == 0) {
                const long long nx = (long long)__hip_atomic_load(next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const long long fin = (long long)__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                stop = nx >= total && total - fin <= handoff ? 1 : 0;
            }
            stop = uniform(stop);
            if (stop) want = false;
            const unsigned long long w = __ballot(want);
            bool have = false;
            if (w != 0ull) {
                const int first = __ffsll((long long)w) - 1;
                unsigned long long base = 0ull;
                if (lane == first) base = atomicAdd(next, (unsigned long long)__popcll(w));
                base = __shfl(base, first);
                const unsigned long long below = lane ? (w & (~0ull >> (64 - lane))) : 0ull;
                const int64_t idx = (int64_t)(base + (unsigned long long)__popcll(below));
                have = want && idx < total;
                if (slot_lane) gidx[f] = have ? supply_frame(st, frame0, idx) : -1ll;
                if (want) {
                    livel[f] = have ? 1 : 0;
                    freshl[f] = have ? 1 : 0;
                    itl[f] = 0;
                }
            }
            const bool gen = __ballot(have) != 0ull;
            want = false;
            const unsigned long long any = __ballot(slot_lane && livel[f] != 0);
            const bool go = any != 0ull && !stop;
            if (!go && slot_lane) {  // the slots' state, in the split path's terms
                const int fr = tile * kTile + lane64;
                st.done[fr] = livel[f] != 0 ? 0 : 1;
                st.iters[fr] = itl[f];
                st.fresh[fr] = freshl[f];
                st.refill[fr] = 0;
            }
            if (lane == 0) {
                flags[2 * kSR + 1] = go ? 1 : 0;
                nref = go && gen ? 1 : 0;
            }
        }
        __syncthreads();
        if (!flags[2 * kSR + 1]) break;  // supply exhausted, every slot drained
        // the new frames, generated by the whole workgroup (u bits staged in
        // zb, which is zero here and again after)
        if (nref) gen_slots<F>(g, st, tile, sub * F, gidx, zb, seed, snr_point, sigma);
        c.live = livel[f] != 0;
        c.fresh = freshl[f] != 0;
        c.ep0 = sub_epoch0(pass, m);
        double tA[K], tB[K];
        bool yA = false, yB = false;
        if (m > 0) {
            sub_stage_commit(c, 0, sub_stage_issue(c, 0));
            yA = sub_p1<Q>(c, 0, sub_chunk(row_ptr, 0, wave, Q), tA);
        }
        for (int r = 0; r <= m; r += 2) {
            sub_body<Q>(c, r, m, tA, yA, tB, yB);
            if (r + 1 <= m) sub_body<Q>(c, r + 1, m, tB, yB, tA, yA);
        }
        __syncthreads();
        sub_p3_reset(c.p3row);

        int my_cnt = 0;
        for (int col = me; col < g.k; col += nthr) {
            double *sp = c.S + (size_t)col * F;
            const double Sj = *sp;
            *sp = 0.0;
            const double chj = *sub_c(c, col);
            const double Lj = chj + Sj;  // channel added after the sum (:173,185)
            if (nllr) {
                const double ap = ld_l2(sub_l(c, col));  // previous L (= ch on a frame's first pass)
                my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
            }
            if (c.live) *sub_l(c, col) = Lj;
            if (!(Lj < 0.0)) atomicOr(zb + (col >> 5) * F + f, 1u << (col & 31));
        }
        if (nllr && my_cnt) atomicAdd(cntl + f, my_cnt);
        __syncthreads();

        uint32_t acc = 0u;  // syndrome (:191-204)
        for (int r = me; r < m; r += nthr) {
            const uint32_t *ar = g.a_packed + (size_t)r * kw;
            uint32_t par = ib[(r >> 5) * F + f] >> (r & 31);
            for (int w = 0; w < kw; ++w) par += __builtin_popcount(ar[w] & zb[w * F + f]);
            acc |= par & 1u;
        }
        if (acc) atomicOr((uint32_t *)bad + f, 1u);
        __syncthreads();

        if (wave == 0) {  // per-slot exits and counters (vn_kernel's stream variant)
            unsigned long long cv[7] = {0, 0, 0, 0, 0, 0, 0};
            bool fin = false;
            if (slot_lane && c.live) {
                const int it = itl[f];
                const bool ok = bad[f] == 0;  // Result.OK at this iteration (:231-241)
                fin = ok || it == max_iter - 1;  // else DATA_TRANSFER_NOT_OK (:244-253)
                if (fin) {
                    int err = 0;
                    if (!ok)  // main.py:130-138: u vs z^1 of a failed frame
                        for (int w = 0; w < kw; ++w) err += __builtin_popcount(Ut[w * kTile] ^ zb[w * F + f]);
                    cv[0] = 1;
                    cv[1] = ok ? 0 : 1;
                    cv[2] = (unsigned long long)err;
                    cv[3] = ok ? (unsigned long long)it : 0;
                    cv[4] = ok ? 1 : 0;
                    cv[5] = nllr ? (unsigned long long)cntl[f] : 0;
                    cv[6] = (unsigned long long)(it + 1);
                    livel[f] = 0;
                    want = true;
                } else {
                    itl[f] = it + 1;
                }
                freshl[f] = 0;
            }
            if (__ballot(fin) != 0ull) {
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const unsigned long long sm = wave_sum(cv[i]);
                    if (lane == 0 && sm) atomicAdd(&ctr[i], sm);
                }
            }
            if (slot_lane) {
                bad[f] = 0;
                cntl[f] = 0;
            }
        }
        __syncthreads();  // wave 0 has read zb (error bits) before it is cleared
        for (int i = threadIdx.x; i < (kw + mw) * F; i += blockDim.x) zb[i] = 0u;
        __syncthreads();
    }
    count_rare_rows(st, c.tseq, kSW);
}

template <int Q>
size_t sub_lds_bytes_q(const DevGraph &g) {
    constexpr int F = SubCfg<Q>::F, K = SubCfg<Q>::K;
    if (!g.std_form || !g.a_packed || g.k <= 0 || g.max_row_deg > kSW * Q * K || Q * K > 64 || g.n > 65535)
        return 0;
    const size_t b = sub_layout(g.k, g.m, F).total;
    return b <= kSubLdsMax ? b : 0;
}

}  // namespace

// Frames per workgroup of the sub-tile decoder for this graph: 16, or 0
// (does not apply).
int sub_frames(const DevGraph &g) { return sub_lds_bytes_q<4>(g) ? 16 : 0; }
size_t sub_lds_bytes(const DevGraph &g) { return sub_lds_bytes_q<4>(g); }

hipError_t launch_tile_sub_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                                  int snr_point, double sigma, int64_t frame0, int64_t total,
                                  unsigned long long *next, unsigned long long *ctr, int64_t handoff, hipStream_t s) {
    const size_t lds = sub_lds_bytes_q<4>(g);
    // the 16-frame form only (+ static LDS: 2 x 16 ints, 16 frame indices, the refill flag)
    if (!lds || !g.a_packed || !st.ubits || 2 * st.ntiles > st.nslots ||
        lds + 2 * 16 * sizeof(int) + 16 * sizeof(long long) + 16 > kSubLdsMax)
        return hipErrorInvalidValue;
    tile_sub_stream_kernel<4><<<st.ntiles * 4, 64 * kSW, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx, g.row_ptr,
                                                                   kAtanhCoef, seed, snr_point, sigma, frame0, total,
                                                                   next, ctr, handoff);
    return hipGetLastError();
}

hipError_t launch_tile_sub(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s) {
    const size_t lds = sub_lds_bytes(g);
    if (!lds || 2 * st.ntiles > st.nslots) return hipErrorInvalidValue;  // two rare-row buffers per workgroup
    tile_sub_kernel<4><<<st.ntiles * 4, 64 * kSW, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx, g.row_ptr,
                                                            kAtanhCoef);
    return hipGetLastError();
}

}  // namespace ldpc
