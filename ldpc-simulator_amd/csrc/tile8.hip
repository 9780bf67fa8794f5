// tile8.hip -- the tile-resident parity decoder of the WiMAX 2304 codes,
// 8 frames per workgroup (gfx950).
//
// Reference: python_ldpc_app/spa_decoder.py:63-280 (SPA_Decoder.decode): per
// check row r (:112-168) t_e = tanh(M_e/2) clipped, P = t_0 * t_1 * ... left to
// right in ascending column order, E_e = 2 atanh(clip(P / t_e)); per column
// (:173-185) S_j = ((0 + E_r0j) + E_r1j) + ... rows ascending, L_j = ch_j + S_j;
// hard decision, syndrome on z^1 and early termination (:188-253); M = L - E
// (:260-268).  Every fp64 operation is the reference's, in its order.
//
// Why 8 frames: the column sums S of a workgroup's frames must sit in LDS
// (k x F x 8 B) and the posteriors L of the A columns are gathered by every
// edge.  With F = 8, wimax_2304_0.5 keeps BOTH in LDS (S and L_A: 2 x 72 KB),
// so the only global traffic left in the row loop is the message stream E
// (read once, written once per iteration: the algorithmic 16 B per edge) and
// one identity-column posterior per row; the r3/4 codes (k = 1728) keep S in
// LDS (108 KB) and gather L from L2 (108 KB per workgroup: 3.5 MB per XCD,
// L2-resident).  Registers hold 3 rows of t (pipeline depth D = 3) and the
// next row's E_old, prefetched one row ahead.  E is laid out in 8-frame blocks
// (DevGraph::ef = 8, spa_device.h e_base) so a lane group's 8 frames of one
// edge are 64 contiguous bytes and two consecutive edges share a cache line.
//
// Mapping: lane = j * 8 + f (lane group j = 0..7, frame f).  A row of an
// [A | I_m] graph is its A edges and, last, the identity column k + r.  The A
// edges are split into 16 contiguous wavefront chunks (wavefront w: positions
// [w*C, w*C + C), C = ceil((deg-1)/16): the host-built P3 order table p3dep8
// assumes this chunking) and a chunk into 8 contiguous lane-group pieces of
// CS = ceil(C/8) edges (slot i of group j = position j*CS + i).  The product
// of the A edges crosses lane groups inside a wavefront by DPP row shifts and
// permlane swaps (VALU only, branch-free) and wavefronts through an LDS slot +
// epoch flag; the identity edge belongs to one wavefront (t_id in P1, E_id and
// L_id in P3: wavefront 0 at D = 3, where it otherwise waits longest for the
// chain; the last one at D = 2),
// and every P3 takes P = P_A * t_id: the reference's left-to-right order.
//
// Per wavefront, body(r) = prefetch(r+1), hop(r), P3(r-D+1), P1(r+1):
//   hop(r)     this wavefront's piece of row r's left-to-right product;
//   P3(r')     E_new = 2 atanh(clip(P/t)), stored; S_col += E_new, after the
//              wavefronts whose column spans overlap finished P3(r'-1);
//   P1(r+1)    M = L[col] - E_old, t = tanh(M/2) (clipped).
// D = 3 gives a row's chain two bodies to cross all 16 wavefronts before its
// P3 needs the final product.
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

constexpr int kW8 = kSubWaves;  // 16 wavefronts per workgroup (p3dep chunking)
constexpr int kF8 = 8;          // frames per workgroup
constexpr int kQ8 = 8;          // lane groups per wavefront
constexpr int kSR8 = 8;         // chain slots (>= 2 D: a slot is reused only after every P3 of its row)
constexpr size_t kLds8Max = 163840;
// -DLDPC_T8_TIMERS: diagnostic build (never the product) -- s_memtime phase
// timers per wavefront, printed for two workgroups at the end of the launch.
#ifdef LDPC_T8_TIMERS
#define T8_NT 9  // hop wait, hop, P3 chain wait, P3 math+stores, P3 order wait, P3 S adds, P1, prefetch, rows
#define T8_STAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define T8_ADD(c, i, a, b) ((c).tm[i] += (b) - (a))
#else
#define T8_STAMP(v)
#define T8_ADD(c, i, a, b)
#endif

// logical wavefront (chunk position) of hardware wavefront hw: the four
// wavefronts of one SIMD take four consecutive chunk positions (as tile_sub.hip)
__device__ __forceinline__ int t8_wave(int hw) { return (hw & 3) * 4 + (hw >> 2); }

// Global accesses go through buffer resources built from wave-uniform bases
// (this workgroup's E block, its tile's L / ch): a 32-bit per-lane voffset,
// the base in SGPRs -- the compiler cannot hoist 64-bit per-lane pointers
// out of the row loop (they spilled, and a scratch reload's vmcnt(0) drained
// the prefetched E_old).  NT = non-temporal (the message stream).
typedef unsigned int t8u2 __attribute__((ext_vector_type(2)));
constexpr int kNT = 2;
constexpr int kEStAux = kNT;  // E_new stores nt (sc1 write-through measured slower: 0.350 vs 0.362, profiles/r4b_ab)
// a voffset past every buffer's num_records: the hardware drops such a store
// (and a load returns 0) -- masked stores without a branch
constexpr uint32_t kOOB = 0xfffffff0u;
template <int AUX = 0>
__device__ __forceinline__ double t8_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
}
template <int AUX = 0>
__device__ __forceinline__ void t8_st(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(t8u2, v), r, off, 0, AUX);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t t8_rsrc(const void *base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)min(bytes, (size_t)0x7fffffff),
                                            0x00020000);
}

struct T8Layout {
    size_t S, LA, math, slot, zb, ib, lane_i, flags, dummy, cidx, total;
};
// R: rows of staged column indices per wavefront (D + 1: P3's row r-D+2 ..
// the staged row r+2 of body(r+1))
__host__ __device__ inline T8Layout t8_layout(int k, int m, int K, bool la, int R, int ns = kSR8) {
    T8Layout t;
    size_t o = 0;
    t.S = o;  // [k][8] column sums
    o = al16(o + (size_t)k * kF8 * sizeof(double));
    t.LA = o;  // [k][8] posteriors of the A columns (previous iteration)
    if (la) o = al16(o + (size_t)k * kF8 * sizeof(double));
    t.math = o;
    o = al16(o + sizeof(MathLds));
    t.slot = o;  // [ns][8] chain slots, then [ns][8] t of the identity edge
    o = al16(o + 2 * (size_t)ns * kF8 * sizeof(double));
    t.zb = o;  // [kw][8] z^1 bits of the A columns
    o = al16(o + (size_t)((k + 31) / 32) * kF8 * sizeof(uint32_t));
    t.ib = o;  // [mw][8] z^1 bits of the identity columns
    o = al16(o + (size_t)((m + 31) / 32) * kF8 * sizeof(uint32_t));
    t.lane_i = o;  // bad[8], nllr count[8], live[8], it[8], fresh[8]
    o = al16(o + 5 * (size_t)kF8 * sizeof(int));
    t.flags = o;  // chain flag[ns], tiny[ns], tiny sequence, running, p3row[16]
    o = al16(o + (2 * (size_t)ns + 2 + kW8) * sizeof(int));
    t.dummy = o;  // [8] target of masked-off S updates
    o = al16(o + (size_t)kF8 * sizeof(double));
    t.cidx = o;  // [R][16][8*K] uint16 column indices, one wavefront chunk per row
    o = al16(o + (size_t)R * kW8 * kQ8 * K * sizeof(uint16_t));
    t.total = o;
    return t;
}

// chain slots (rows) and index-ring rows of a variant: the row form kSR8 and
// D + 1; the pair form 2 per chain slot (tp_slots) and 2 ring rows
__host__ __device__ constexpr int t8_ns(bool pair, int D) { return pair ? 2 * 4 : kSR8; }
__host__ __device__ constexpr int t8_ring(bool pair, int D) { return pair ? 2 : D + 1; }

// deg: the whole row; the chunks cover its A edges (all but the last, the
// identity column k + r at edge eid = beg + deg - 1).
struct T8Chunk {
    int deg, beg, c0, cnt, CS;
};
__device__ __forceinline__ T8Chunk t8_chunk(const int *__restrict__ row_ptr, int r, int wave) {
    T8Chunk c;
    c.beg = row_ptr[r];
    c.deg = row_ptr[r + 1] - c.beg;
    const int da = max(c.deg - 1, 0);
    const int C = (da + kW8 - 1) / kW8;
    c.c0 = c.beg + wave * C;
    c.cnt = max(0, min(da - wave * C, C));
    c.CS = (C + kQ8 - 1) / kQ8;
    return c;
}

template <int K>
struct T8Ctx {
    const int *__restrict__ col_idx;
    const int *__restrict__ row_ptr;
    const int *p3dep;
    // buffer resources (uniform) + per-lane byte offsets eo8 (E block: f * 8)
    // and lo8 (L / ch: (sub*8 + f) * 8)
    __amdgpu_buffer_rsrc_t rE;  // this workgroup's E block: edge e, frame f at e*64 + f*8
    __amdgpu_buffer_rsrc_t rL, rC;  // the tile's L / ch: column c at c*512 + lo8
    uint32_t eo8, lo8;
    double *Tb;      // rare-row scratch of this workgroup, position p at [p * 8]; two buffers
    size_t tbuf;     // doubles between them (rare rows alternate: tile_kernels.hip)
    double *S;       // LDS, column c at [c * 8] (this lane's frame added)
    double *LA;      // LDS, same indexing (null: L gathered from global)
    double *dummy;   // LDS, this lane's frame
    double *slot;    // LDS, chain slot s at [s * 8]; t of row s's identity edge at [(kSR8 + s) * 8]
    uint32_t *ib;    // LDS, word w at [w * 8]
    uint16_t *cidx;  // LDS, this wavefront's ring: row slot q, position p at [q * 16 * 8K + p]
    int *flag, *tinyf, *tseq, *p3row;
    LdsTanh ttab;
    LdsAtanh ltab;
    AtanhCoef ac;   // kernel-argument coefficients (when coef_arg)
    bool coef_arg;  // P3 uses ac instead of coef_load() (compile-time per kernel)
    int m, k, wave, j, f, nnz;
    int h;  // pair form: this lane's row of the pair (lane = h*32 + j*8 + f); 0 otherwise
    int ep0;
    bool first, live, fresh;
    int ntiny;
    int R;       // ring rows
    int ns;      // chain slots (rows; pair form: 2 per pair)
    int idwave;  // the wavefront that owns the identity edge
#ifdef LDPC_T8_TIMERS
    uint64_t tm[T8_NT];
#endif
};

// This lane's edge count in chunk rc.
template <int K>
__device__ __forceinline__ int t8_nj(const T8Ctx<K> &c, const T8Chunk &rc) {
    return max(0, min(rc.cnt - c.j * rc.CS, rc.CS));
}
// Byte offset (from c.Eu) of this lane's slot 0 in chunk rc; slot i at + i * 64.
// Slots past the lane's piece read other edges (or the allocation's
// kEPadEdges slack) and are discarded.
template <int K>
__device__ __forceinline__ uint32_t t8_eoff(const T8Ctx<K> &c, const T8Chunk &rc) {
    return ((uint32_t)(rc.c0 + c.j * rc.CS) << 6) + c.eo8;
}
template <int K>
__device__ __forceinline__ uint32_t t8_es(const T8Ctx<K> &c, uint32_t off, int i) {
    return off + (uint32_t)i * (kF8 * sizeof(double));
}

// Staging of row q's column indices into the ring: issue (one index per lane,
// lanes < the chunk size), commit once the wavefront has waited anyway.
template <int K>
__device__ __forceinline__ int t8_stage_issue(const T8Ctx<K> &c, int q) {
    // always one load of an in-range edge (see t8_prefetch)
    const T8Chunk rc = t8_chunk(c.row_ptr, min(q, c.m - 1), c.wave);
    const int L = threadIdx.x & 63;
    return c.col_idx[min(max(rc.c0 + min(L, rc.cnt - 1), 0), c.nnz - 1)];
}
template <int K>
__device__ __forceinline__ void t8_stage_commit(const T8Ctx<K> &c, int q, int v) {
    if (q >= c.m) return;
    constexpr int W = kQ8 * K;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if ((int)(threadIdx.x & 63) < W) c.cidx[(q % c.R) * kW8 * W + (threadIdx.x & 63)] = (uint16_t)v;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int K>
__device__ __forceinline__ const uint16_t *t8_lcols(const T8Ctx<K> &c, int r, const T8Chunk &rc) {
    return c.cidx + (r % c.R) * kW8 * kQ8 * K + c.j * rc.CS;
}

// Next row's loads that do not depend on the staged indices: E_old of this
// lane's K slots and the identity column's posterior (L[k+r], or ch[k+r] on
// iteration 0 / a fresh frame's first pass).
template <int K>
struct T8Pre {
    double eo[K];
    double lid, eid;  // wavefront 0: the identity column's posterior and E_old
};
// (iteration 0 and a fresh streaming frame's lanes form M = L - 0.0 == L and
// read no E_old: exec-masked)
// Every load is issued unconditionally, masked ones at kOOB (the buffer
// returns 0 without a memory request): with loads under branches the
// compiler's vmcnt counts were conservative and P1 waited for the previous
// row's E_new stores before its first request (tile_sub.hip, round 5).
template <int K>
__device__ __forceinline__ void t8_prefetch(const T8Ctx<K> &c, int r, T8Pre<K> &p) {
    const T8Chunk rc = t8_chunk(c.row_ptr, r, c.wave);
    const bool noE = c.first || c.fresh;
    const uint32_t eoff = t8_eoff(c, rc);
#pragma unroll
    for (int i = 0; i < K; ++i) p.eo[i] = t8_ld<kNT>(c.rE, (rc.cnt > 0 && !noE) ? t8_es(c, eoff, i) : kOOB);
    // identity edge (a fresh streaming frame has L = ch: gen_slots)
    const bool id = c.wave == c.idwave && rc.deg > 0;
    p.lid = t8_ld(c.first ? c.rC : c.rL, id ? ((uint32_t)(c.k + r) << 9) + c.lo8 : kOOB);
    p.eid = t8_ld<kNT>(c.rE, (id && !noE) ? ((uint32_t)(rc.beg + rc.deg - 1) << 6) + c.eo8 : kOOB);
}

// P1: t = tanh((L[col] - E_old)/2) for this lane's slots, columns into col[];
// returns whether some lane's own edge has |t| <= 1e-10 (:159).  Every slot is
// evaluated (branch-free): slots past the piece hold valid data and end as 1.0
// -- except slot K-1 of a row whose pieces are shorter than K (wave-uniform;
// 561 of the 576 rows of wimax_2304_0.75A have CS = 7 of K = 8), which takes
// 1.0 without its tanh (+3 %, profiles/r4b_ab).  P3 adds each slot's E_new
// into its column sum with one ds_add_f64 (tile_sub.hip: the same IEEE add,
// no read round trip) and, on saturated rows, reuses slot 0's E_new (t8_p3).
template <int K, bool LA>
__device__ __forceinline__ void t8_p1_slots(const T8Ctx<K> &c, int r, const T8Chunk &rc, const T8Pre<K> &pre,
                                            double (&t)[K], bool &tiny, bool skip_last) {
    const int nj = t8_nj(c, rc);
    const int njt = c.live ? nj : 0;  // the |t| <= 1e-10 vote: frame-less lanes abstain
    const uint16_t *lc = t8_lcols(c, r, rc);
    double Lv[K];
    int col[K];
#pragma unroll
    for (int i = 0; i < K; ++i) col[i] = lc[i];
    if constexpr (LA) {
#pragma unroll
        for (int i = 0; i < K; ++i) Lv[i] = c.LA[(size_t)col[i] * kF8];
    } else {
        const __amdgpu_buffer_rsrc_t rs = c.first ? c.rC : c.rL;  // iteration 0: M = ch (:85-90)
#pragma unroll
        for (int i = 0; i < K; ++i) Lv[i] = t8_ld(rs, ((uint32_t)col[i] << 9) + c.lo8);
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (i == K - 1 && skip_last) {  // wave-uniform: no piece reaches slot K-1 in this row
            t[i] = 1.0;
            continue;
        }
        // :85-90 / :260-268 (eo = 0.0 on iteration 0; a fresh streaming frame M = L)
        const double M = c.fresh ? Lv[i] : Lv[i] - pre.eo[i];
        const double tv = tanh_half_clipped(M, c.ttab);  // :138-146 (spa_math.h)
        tiny |= i < njt && !(fabs(tv) > kTiny);
        t[i] = i < nj ? tv : 1.0;  // past the piece: an exact no-op in the product
    }
}

template <int K, bool LA>
__device__ __forceinline__ bool t8_p1(const T8Ctx<K> &c, int r, const T8Pre<K> &pre, double (&t)[K]) {
    bool tiny = false;
    const int sv = t8_stage_issue(c, r + 1);
    const T8Chunk rc = t8_chunk(c.row_ptr, r, c.wave);
    // no branch on rc.cnt (its loads stay unconditional: t8_prefetch); an
    // empty chunk has nj = 0, so every slot ends as 1.0 (the staged indices
    // are valid columns)
    t8_p1_slots<K, LA>(c, r, rc, pre, t, tiny, rc.CS < K);
    if (c.wave == c.idwave && rc.deg > 0) {  // the identity edge: t_id, published for every P3 of row r
        const double M = c.fresh ? pre.lid : pre.lid - pre.eid;
        const double tv = tanh_half_clipped(M, c.ttab);
        tiny |= c.live && !(fabs(tv) > kTiny);
        if (c.j == 0) c.slot[(kSR8 + (r & (kSR8 - 1))) * kF8] = tv;
    }
    t8_stage_commit(c, r + 1, sv);
    return __ballot(tiny) != 0ull;
}

// Lane-group hand-over: group jj's value into group jj+1 (lane = group*8 + f;
// groups 2a, 2a+1 are the halves of DPP row a).  Even jj: row_shr:8 inside the
// row; odd jj: row_ror:8 (upper half to lower half), then row a -> a+1 by
// v_permlane16/32_swap (tile_sub.hip group_up4).
__device__ __forceinline__ uint32_t t8_p16(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t t8_p32(uint32_t x, int which) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return which ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t t8_up(uint32_t x, int jj) {
    if ((jj & 1) == 0) return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x118, 0xf, 0xf, false);
    x = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x128, 0xf, 0xf, false);
    return (jj >> 1) == 1 ? t8_p16(t8_p32(x, 0), 1) : t8_p16(x, 0);
}
__device__ __forceinline__ double t8_group_up(double v, int jj) {
    const uint64_t u = dbits(v);
    const uint32_t lo = t8_up((uint32_t)u, jj), hi = t8_up((uint32_t)(u >> 32), jj);
    return dfrom(((uint64_t)hi << 32) | lo);
}

// hop: this wavefront's chunk of row r's left-to-right product (:151-152).
template <int K>
__device__ __forceinline__ void t8_hop(T8Ctx<K> &c, int r, const double (&t)[K], bool tiny) {
    const T8Chunk rc = t8_chunk(c.row_ptr, r, c.wave);
    if (rc.deg == 0) return;  // spa_decoder.py:115-122
    const int s = r & (kSR8 - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    double *sl = c.slot + s * kF8;
    double P = 1.0;  // 1.0 * t0 == t0 exactly
    T8_STAMP(h0);
    if (c.wave != 0) {
        wait_flag<false>(c.flag + s, ep + c.wave);
        P = *sl;
    }
    T8_STAMP(h1);
    T8_ADD(c, 0, h0, h1);
    __builtin_amdgcn_s_setprio(2);
    if (rc.cnt > 0) {
        // branch-free: every lane group multiplies all K slots (slots past its
        // piece, and every slot of a group past the chunk, hold 1.0: exact
        // no-ops), so the product ends in group 7 whatever the chunk's length
        if (K > 1 && rc.CS < K) {  // slot K-1 holds 1.0 in every group: skip it
#pragma unroll
            for (int jj = 0; jj < kQ8; ++jj) {
#pragma unroll
                for (int i = 0; i < K - 1; ++i) P = P * t[i];
                if (jj + 1 < kQ8) P = t8_group_up(P, jj);
            }
        } else {
#pragma unroll
            for (int jj = 0; jj < kQ8; ++jj) {
#pragma unroll
                for (int i = 0; i < K; ++i) P = P * t[i];
                if (jj + 1 < kQ8) P = t8_group_up(P, jj);
            }
        }
    }
    if ((threadIdx.x & 63) == 0) {
        if (c.wave == 0)
            lds_st(c.tinyf + s, tiny ? 1 : 0);
        else if (tiny)
            lds_st(c.tinyf + s, 1);
    }
    if (c.j == kQ8 - 1) *sl = P;
    lds_release();
    if ((threadIdx.x & 63) == 0) lds_st(c.flag + s, ep + c.wave + 1);
    __builtin_amdgcn_s_setprio(0);
    T8_STAMP(h2);
    T8_ADD(c, 1, h1, h2);
}

// P3 of row r: E_new of this lane's slots (:159-168), stored; then, after
// row r-1's P3 by the wavefronts whose column spans overlap this chunk's
// (p3dep, ldpc_api.cpp sub_p3_deps: every column's additions stay rows
// ascending), S_col += E_new; the identity column's posterior and z^1 bit.
// p3row[v] = 1 + the last row of this pass whose P3 wavefront v finished.
template <int K>
__device__ __forceinline__ void t8_p3(T8Ctx<K> &c, int r, double (&t)[K]) {
    const T8Chunk rc = t8_chunk(c.row_ptr, r, c.wave);
    if (rc.deg == 0) {
        if ((threadIdx.x & 63) == 0) lds_st(c.p3row + c.wave, r + 1);
        return;
    }
    const int s = r & (kSR8 - 1);
    const int ep = ((c.ep0 + r) & 0x3ffffff) * 32;
    const bool idw = c.wave == c.idwave;  // holds the identity edge
    const double chI = t8_ld(c.rC, idw ? ((uint32_t)(c.k + r) << 9) + c.lo8 : kOOB);  // for L = ch + (0 + E)
    int col[K];  // staged indices (ring row r is live until body(r + D - 1) ends)
    {
        const uint16_t *lc = t8_lcols(c, r, rc);
#pragma unroll
        for (int i = 0; i < K; ++i) col[i] = lc[i];
    }
    T8_STAMP(q0);
    wait_flag<false>(c.flag + s, ep + kW8);  // row r's A product is complete
    T8_STAMP(q1);
    T8_ADD(c, 2, q0, q1);
    const bool tiny_row = uniform(lds_ld(c.tinyf + s)) != 0;
    const AtanhCoef ac = c.coef_arg ? c.ac : coef_load();  // scalar loads for this P3 only (cn_common.h)
    const int nj = t8_nj(c, rc);
    const double tI = c.slot[(kSR8 + s) * kF8];
    const double P = c.slot[s * kF8] * tI;  // (t_0 * ... * t_{deg-2}) * t_id: left to right (:151-152)
    double EI = 0.0;
    if (!tiny_row) {
        // q = P/t, then E_new = 2 atanh(clip(q)) (:159-168), or 2q when every
        // quotient of the wavefront is below 2^-27 (exact: spa_math.h
        // kAtanhIdent), decided slot by slot
        const double lim = c.live ? kAtanhIdent : INFINITY;  // frame-less lanes do not vote
        auto en = [&](double q) {
            return __ballot(!(fabs(q) < lim)) == 0ull ? 2.0 * q : 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
        };
        if (div_nr_ok(c.live ? P : 1.0)) {  // the IEEE quotient without its scaling steps (cn_common.h)
            if (rc.cnt > 0) {
                if (K == 8) {  // the r3/4 form (the L_A form spills with it)
                    // Saturated rows (config 4's 3.5 and 4 dB points: 99.8 % of
                    // the edges have |M| >= 35, t = +-CL) give most slots one
                    // quotient magnitude.  atanh_f(clip_cl(q)) is odd in q and
                    // 2q == 2 atanh_f(clip_cl(q)) below 2^-27, so a slot where
                    // every lane's |q| equals its slot-0 |q| takes slot 0's
                    // E_new with its own sign: the same function of the same
                    // argument (bit for bit; the key only decides how often it
                    // hits), one atanh per lane and row instead of one per slot.
                    // Lanes that do not vote (frame-less, past the piece) keep
                    // values nothing stores or uses.
                    double key = 0.0;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        if (i < rc.CS) {
                            const double q = div_nr(P, t[i]);
                            if (i == 0) key = fabs(q);
                            if (__ballot(!(fabs(q) < lim)) == 0ull)
                                t[i] = 2.0 * q;
                            else if (i > 0 && __ballot(c.live && i < nj && fabs(q) != key) == 0ull)
                                t[i] = dfrom((dbits(t[0]) & 0x7fffffffffffffffull) | (dbits(q) & 0x8000000000000000ull));
                            else
                                t[i] = 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
                        }
                                }
                } else {
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        if (i < rc.CS) t[i] = en(div_nr(P, t[i]));
                                }
                }
            }
            if (idw) EI = en(div_nr(P, tI));
        } else {
            if (rc.cnt > 0) {
#pragma unroll
                for (int i = 0; i < K; ++i)
                    if (i < rc.CS) t[i] = en(P / t[i]);
            }
            if (idw) EI = en(P / tI);
        }
    } else {
        // rare: q = in-order product of the others (np.prod(np.delete(...)),
        // :164) for an edge with |t| <= 1e-10; t parked at row positions (the
        // identity edge at deg-1).  Every wavefront takes part in the count.
        const int pos0 = rc.c0 + c.j * rc.CS - rc.beg;
        double *tb = c.Tb + (c.ntiny & 1) * c.tbuf;  // the next rare row parks in the other buffer
        if (rc.cnt > 0) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < nj) tb[(size_t)(pos0 + i) * kF8] = t[i];
        }
        if (idw && c.j == 0) tb[(size_t)(rc.deg - 1) * kF8] = tI;
        __builtin_amdgcn_s_waitcnt(0);  // scratch stores have reached L2
        c.ntiny += 1;
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c.tseq, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_flag<false>(c.tseq, c.ntiny * kW8);
        auto others = [&](int pos) {
            double q = 1.0;
            bool fst = true;
            for (int p = 0; p < rc.deg; ++p) {
                if (p == pos) continue;
                const double t2 = ld_l2(tb + (size_t)p * kF8);
                q = fst ? t2 : q * t2;
                fst = false;
            }
            return q;
        };
        if (rc.cnt > 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) {
                if (i < rc.CS) {
                    const double ti = t[i];
                    const double q = (fabs(ti) > kTiny || i >= nj) ? P / ti : others(pos0 + i);
                    t[i] = 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
                }
            }
        }
        if (idw) {
            const double q = fabs(tI) > kTiny ? P / tI : others(rc.deg - 1);
            EI = 2.0 * atanh_f(clip_cl(q), c.ltab, ac);
        }
    }
    {  // slots past the piece (and frames that stopped) store out of range: dropped (no branch)
        const uint32_t eoff = t8_eoff(c, rc);
#pragma unroll
        for (int i = 0; i < K; ++i) t8_st<kEStAux>(c.rE, (i < nj && c.live) ? t8_es(c, eoff, i) : kOOB, t[i]);
        t8_st<kEStAux>(c.rE, (c.live && idw && c.j == 0) ? ((uint32_t)(rc.beg + rc.deg - 1) << 6) + c.eo8 : kOOB,
                       EI);
    }
    // S order: row r-1's P3 by the overlapping wavefronts
    T8_STAMP(q2);
    T8_ADD(c, 3, q1, q2);
    if (r > 0) {
        const int d = ld_table(c.p3dep, r * kW8 + c.wave);
        for (int v = d & 0xff; v <= (d >> 8); ++v) wait_ge<false>(c.p3row + v, r);
    }
    T8_STAMP(q3);
    T8_ADD(c, 4, q2, q3);
    if (rc.cnt > 0) {
        // S_col += E_new, rows ascending; a lane's slots never share a column
        // within a row, so all reads, all adds, all writes (one LDS round trip)
        double *sp[K];
#pragma unroll
        for (int i = 0; i < K; ++i) sp[i] = i < nj ? c.S + (size_t)col[i] * kF8 : c.dummy;
#pragma unroll
        for (int i = 0; i < K; ++i)  // one ds_add_f64 per slot; past the piece: `dummy`
            __hip_atomic_fetch_add(sp[i], t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    {  // identity column: L = ch + (0 + E) (:173-185)
        const bool own = idw && c.j == 0;
        const double Lj = chI + (0.0 + EI);
        t8_st(c.rL, (own && c.live) ? ((uint32_t)(c.k + r) << 9) + c.lo8 : kOOB, Lj);
        if (own && !(Lj < 0.0)) atomicOr(c.ib + (r >> 5) * kF8, 1u << (r & 31));
    }
    lds_release();  // this row's S additions before the count
    if ((threadIdx.x & 63) == 0) lds_st(c.p3row + c.wave, r + 1);
    T8_STAMP(q4);
    T8_ADD(c, 5, q3, q4);
}

// body(r) with t/col buffers B (hop), B+1 mod D (P3 of row r-D+1, then P1 of r+1)
// LA variants prefetch the next row's E_old (and identity loads) before
// hop + P3; the L-gathering variant (8 slots per lane) has no registers for
// that and issues them at the start of P1.
template <int K, bool LA, int D, int B>
__device__ __forceinline__ void t8_body(T8Ctx<K> &c, int r, double (&t)[D][K], bool (&y)[D]) {
    constexpr int N = (B + 1) % D;
    T8Pre<K> pre;
    T8_STAMP(a0);
    if (LA && r + 1 < c.m) t8_prefetch(c, r + 1, pre);
    T8_STAMP(a1);
    T8_ADD(c, 7, a0, a1);
    if (r < c.m) t8_hop(c, r, t[B], y[B]);
    if (r >= D - 1) t8_p3(c, r - (D - 1), t[N]);
    T8_STAMP(a2);
    if (!LA && r + 1 < c.m) t8_prefetch(c, r + 1, pre);
    if (r + 1 < c.m) y[N] = t8_p1<K, LA>(c, r + 1, pre, t[N]);
    T8_STAMP(a3);
    T8_ADD(c, 6, a2, a3);
}

// One pass over all rows (every P3 done on return, before the barrier).
template <int K, bool LA, int D>
__device__ __forceinline__ void t8_rows(T8Ctx<K> &c) {
    const int m = c.m;
    double t[D][K];
    bool y[D];
    if (m <= 0) return;
    {
        t8_stage_commit(c, 0, t8_stage_issue(c, 0));
        T8Pre<K> pre;
        t8_prefetch(c, 0, pre);
        y[0] = t8_p1<K, LA>(c, 0, pre, t[0]);
    }
    const int last = m + D - 2;  // body(last) runs P3(m-1)
    for (int r = 0; r <= last; r += D) {
        t8_body<K, LA, D, 0>(c, r, t, y);
        if (r + 1 <= last) t8_body<K, LA, D, 1>(c, r + 1, t, y);
        if constexpr (D == 3)
            if (r + 2 <= last) t8_body<K, LA, D, 2>(c, r + 2, t, y);
    }
}

// ---------------------------------------------------------------------------
// Pair form: TWO rows per wavefront.  lane = h*32 + j*8 + f: half h carries row
// 2q + h of row pair q, in 4 lane groups j of the 8 frames f.  A row's A edges
// are chunked over the 16 wavefronts exactly as above (C = ceil((deg-1)/16):
// p3dep8 applies unchanged) and a chunk over 4 lane-group pieces of
// CS = ceil(C/4) <= K edges, so one wavefront instruction covers 64 lane-edges
// with 4 groups per row -- tile_sub.hip's instruction shape (its 16 frames x 4
// groups) on the 8-frame layout that keeps the column sums AND the A-column
// posteriors in LDS: P1 reads L[col] from LDS instead of gathering it from L2
// (the 8-frame decoder above pays 8 lane groups per row for that, 117 VALU per
// wave slot against tile_sub's 83, profiles/r5a_counters).  Both rows' products
// run in the same instructions: each half hands its running product group to
// group (DPP row_shr / row_ror + permlane16) and wavefront to wavefront through
// its own LDS slot.  P3 adds half 0's E_new (row 2q), publishes, then half 1's
// (row 2q+1) after the overlapping wavefronts' row 2q: the rows-ascending order
// of every column sum.  Pipeline body(q) = hop(q), P3(q-1), P1(q+1); the column
// indices of pair q+1 are staged during P3(q-1) into the ring row P3(q-1) has
// just read (2 ring rows).  Chain slots: kPSR pairs x 2 halves in the same LDS
// as the row form's kSR8 rows.
constexpr int kPQ = 4;    // lane groups per row
// chain slots (pairs) of the pair form: a slot is reused only after every P3
// of its pair (wavefront 0's P1(q) follows its P3(q-2), which waited for every
// wavefront's hop(q-2), i.e. their P3(q-4)); 2 per pair in the layout
template <int D>
__host__ __device__ constexpr int tp_slots() { return 4; }

struct PChunk {
    int deg, beg, c0, cnt, CS;  // this lane's row (per half)
    int cs_max;                 // max CS over the two rows (uniform)
    bool any;                   // some chunk of this wavefront has edges (uniform)
};
template <int K>
__device__ __forceinline__ PChunk tp_chunk(const T8Ctx<K> &c, int q) {
    const int r0 = 2 * q;
    // uniform (scalar) loads; rows >= m are empty
    const int b0 = c.row_ptr[min(r0, c.m)], b1 = c.row_ptr[min(r0 + 1, c.m)], b2 = c.row_ptr[min(r0 + 2, c.m)];
    const int da0 = max(b1 - b0 - 1, 0), da1 = max(b2 - b1 - 1, 0);
    const int C0 = (da0 + kW8 - 1) / kW8, C1 = (da1 + kW8 - 1) / kW8;
    const int n0 = max(0, min(da0 - c.wave * C0, C0)), n1 = max(0, min(da1 - c.wave * C1, C1));
    PChunk rc;
    rc.beg = c.h ? b1 : b0;
    rc.deg = (c.h ? b2 : b1) - rc.beg;
    const int C = c.h ? C1 : C0;
    rc.c0 = rc.beg + c.wave * C;
    rc.cnt = c.h ? n1 : n0;
    rc.CS = (C + kPQ - 1) / kPQ;
    rc.cs_max = (max(C0, C1) + kPQ - 1) / kPQ;
    rc.any = n0 > 0 || n1 > 0;
    return rc;
}
template <int K>
__device__ __forceinline__ int tp_nj(const T8Ctx<K> &c, const PChunk &rc) {
    return max(0, min(rc.cnt - c.j * rc.CS, rc.CS));
}
// ring row q%2: half h's 4K positions at [h * 4K], this lane's slot i at [j*CS + i]
template <int K>
__device__ __forceinline__ const uint16_t *tp_lcols(const T8Ctx<K> &c, int q, const PChunk &rc) {
    return c.cidx + (q & 1) * kW8 * 8 * K + c.h * kPQ * K + c.j * rc.CS;
}
// Staging of pair q's indices: lane L takes position L of both rows' chunks
// (clamped to the chunk's last edge; rows past the chunk: 0).
struct TpStage {
    int v0, v1;
};
template <int K>
__device__ __forceinline__ TpStage tp_stage_issue(const T8Ctx<K> &c, int q) {
    TpStage v{0, 0};
    if (2 * q >= c.m) return v;
    const int r0 = 2 * q;
    const int b0 = c.row_ptr[r0], b1 = c.row_ptr[min(r0 + 1, c.m)], b2 = c.row_ptr[min(r0 + 2, c.m)];
    const int da0 = max(b1 - b0 - 1, 0), da1 = max(b2 - b1 - 1, 0);
    const int C0 = (da0 + kW8 - 1) / kW8, C1 = (da1 + kW8 - 1) / kW8;
    const int n0 = max(0, min(da0 - c.wave * C0, C0)), n1 = max(0, min(da1 - c.wave * C1, C1));
    const int L = threadIdx.x & 63;
    if (n0 > 0) v.v0 = c.col_idx[b0 + c.wave * C0 + min(L, n0 - 1)];
    if (n1 > 0) v.v1 = c.col_idx[b1 + c.wave * C1 + min(L, n1 - 1)];
    return v;
}
template <int K>
__device__ __forceinline__ void tp_stage_commit(const T8Ctx<K> &c, int q, TpStage v) {
    if (2 * q >= c.m) return;
    constexpr int W = kPQ * K;  // positions per row chunk
    const int L = threadIdx.x & 63;
    uint16_t *ring = c.cidx + (q & 1) * kW8 * 8 * K;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (L < W) {
        ring[L] = (uint16_t)v.v0;
        ring[W + L] = (uint16_t)v.v1;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// P1 of pair q: t = tanh((L[col] - E_old)/2) of this lane's slots (L_A from
// LDS); the identity edges' t (idwave) published in the pair's slot.  Returns
// the rows' |t| <= 1e-10 votes: bit h = some live lane of half h.
// this lane's slot i column (the staged ring)
template <int K, int D>
__device__ __forceinline__ int tp_col(const T8Ctx<K> &c, int q, const PChunk &rc, int i) {
    return tp_lcols(c, q, rc)[i];
}
template <int K, int D>
__device__ __forceinline__ int tp_p1(const T8Ctx<K> &c, int q, double (&t)[K]) {
    const PChunk rc = tp_chunk(c, q);
    bool tiny = false;
    const int nj = tp_nj(c, rc);
    const int njt = c.live ? nj : 0;  // frame-less lanes abstain
    if (rc.any) {
        const uint32_t eoff = ((uint32_t)(rc.c0 + c.j * rc.CS) << 6) + c.eo8;
        const bool noE = c.first || c.fresh;  // M = L - 0.0 == L: no E_old
        // E_old straight into t (all slots in flight); L[col] from LDS just
        // before each slot's tanh (short latency: no second array of loads)
#pragma unroll
        for (int i = 0; i < K; ++i) t[i] = noE ? 0.0 : t8_ld<kNT>(c.rE, t8_es(c, eoff, i));
        const bool skip_last = rc.cs_max < K;  // wave-uniform: no piece reaches slot K-1
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if (i == K - 1 && skip_last) {
                t[i] = 1.0;
                continue;
            }
            const double Lc = c.LA[(size_t)tp_col<K, D>(c, q, rc, i) * kF8];  // L[col] (LDS)
            const double M = Lc - t[i];  // :85-90 / :260-268 (t = E_old, or +0.0 on a first pass: M == L bit for bit)
            const double tv = tanh_half_clipped(M, c.ttab);  // :138-146
            tiny |= i < njt && !(fabs(tv) > kTiny);
            t[i] = i < nj ? tv : 1.0;  // past the piece: an exact no-op in the product
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) t[i] = 1.0;
    }
    if (c.wave == c.idwave) {  // the identity edges k + 2q + h (a fresh frame has L = ch: gen_slots)
        const int r = 2 * q + c.h;
        if (rc.deg > 0) {
            const bool noE = c.first || c.fresh;
            const double lid = t8_ld(c.first ? c.rC : c.rL, ((uint32_t)(c.k + r) << 9) + c.lo8);
            const double eid = noE ? 0.0 : t8_ld<kNT>(c.rE, ((uint32_t)(rc.beg + rc.deg - 1) << 6) + c.eo8);
            const double tv = tanh_half_clipped(noE ? lid : lid - eid, c.ttab);
            tiny |= c.live && !(fabs(tv) > kTiny);
            if (c.j == 0) c.slot[(c.ns + (q & (tp_slots<D>() - 1)) * 2 + c.h) * kF8] = tv;
        }
    }
    const unsigned long long b = __ballot(tiny);
    return ((uint32_t)b != 0u ? 1 : 0) | ((b >> 32) != 0ull ? 2 : 0);
}

// hop of pair q: this wavefront's chunks of both rows' left-to-right products.
template <int K, int D>
__device__ __forceinline__ void tp_hop(T8Ctx<K> &c, int q, const double (&t)[K], int tiny) {
    const int s = q & (tp_slots<D>() - 1);
    const int ep = ((c.ep0 + q) & 0x3ffffff) * 32;
    double *sl = c.slot + (s * 2 + c.h) * kF8;
    double P = 1.0;  // 1.0 * t0 == t0 exactly
    T8_STAMP(h0);
    if (c.wave != 0) {
        wait_flag<false>(c.flag + s, ep + c.wave);
        P = *sl;
    }
    T8_STAMP(h1);
    T8_ADD(c, 0, h0, h1);
    __builtin_amdgcn_s_setprio(2);
    if (uniform(tp_chunk(c, q).any ? 1 : 0)) {
        // branch-free: every group multiplies all K slots (1.0-padded: exact
        // no-ops), the running product moves group j -> j+1 inside each half
        // (t8_up's first three steps), so it ends in group 3 of each half
#pragma unroll
        for (int jj = 0; jj < kPQ; ++jj) {
#pragma unroll
            for (int i = 0; i < K; ++i) P = P * t[i];
            if (jj + 1 < kPQ) P = t8_group_up(P, jj);
        }
    }
    if ((threadIdx.x & 63) == 0) {
        if (c.wave == 0) {
            lds_st(c.tinyf + s * 2, tiny & 1);
            lds_st(c.tinyf + s * 2 + 1, tiny >> 1);
        } else {
            if (tiny & 1) lds_st(c.tinyf + s * 2, 1);
            if (tiny & 2) lds_st(c.tinyf + s * 2 + 1, 1);
        }
    }
    if (c.j == kPQ - 1) *sl = P;
    lds_release();
    if ((threadIdx.x & 63) == 0) lds_st(c.flag + s, ep + c.wave + 1);
    __builtin_amdgcn_s_setprio(0);
    T8_STAMP(h2);
    T8_ADD(c, 1, h1, h2);
}

// Row r's S additions may start once the wavefronts whose column spans
// overlap this one's have added row r-1 (p3row[v] = 1 + their last row).
template <int K>
__device__ __forceinline__ void tp_order(const T8Ctx<K> &c, int r) {
    if (r > 0 && r < c.m) {
        const int d = c.p3dep[r * kW8 + c.wave];
        for (int v = d & 0xff; v <= (d >> 8); ++v) wait_ge<false>(c.p3row + v, r);
    }
}

// P3 of pair q: E_new of this lane's slots (:159-168), stored; S_col += E_new
// row 2q then row 2q+1 in the column order; the identity columns' posteriors
// and z^1 bits.  The indices of pair q+2 (staged by the caller) replace this
// pair's ring row once read.
template <int K, int D>
__device__ __forceinline__ void tp_p3(T8Ctx<K> &c, int q, double (&t)[K], TpStage nxt) {
    const PChunk rc = tp_chunk(c, q);
    const int s = q & (tp_slots<D>() - 1);
    const int ep = ((c.ep0 + q) & 0x3ffffff) * 32;
    const int r = 2 * q + c.h;
    const bool idw = c.wave == c.idwave && rc.deg > 0;  // this lane holds its row's identity edge
    double chI = 0.0;
    if (idw) chI = t8_ld(c.rC, ((uint32_t)(c.k + r) << 9) + c.lo8);  // for L = ch + (0 + E)
    // this pair's staged columns; its ring row takes pair q+2's next
    int col[K];
#pragma unroll
    for (int i = 0; i < K; ++i) col[i] = tp_col<K, D>(c, q, rc, i);
    tp_stage_commit(c, q + 2, nxt);  // the ring row is read (in-order LDS of this wavefront)
    T8_STAMP(q0);
    wait_flag<false>(c.flag + s, ep + kW8);  // both rows' A products are complete
    T8_STAMP(q1);
    T8_ADD(c, 2, q0, q1);
    const bool tiny_row = lds_ld(c.tinyf + s * 2 + c.h) != 0;
    const AtanhCoef ac = c.coef_arg ? c.ac : coef_load();  // scalar loads for this P3 only (cn_common.h)
    const bool tiny_any = __ballot(tiny_row) != 0ull;
    const int nj = tp_nj(c, rc);
    const double tI = c.slot[(c.ns + s * 2 + c.h) * kF8];
    const double P = c.slot[(s * 2 + c.h) * kF8] * tI;  // (t_0 * ... * t_{deg-2}) * t_id: left to right
    // E_new stored (slots past the piece and frames that stopped store out of
    // range: dropped); S_col += E_new row 2q then row 2q+1 in the column
    // order; the identity columns.  Called at the end of each branch so the
    // branches' E_new values never merge (a merge cost ~200 spilled VGPRs).
    auto finish = [&](double (&tt)[K], double EI) {
        {  // slots past the piece (and frames that stopped) store out of range: dropped
            const uint32_t eoff = ((uint32_t)(rc.c0 + c.j * rc.CS) << 6) + c.eo8;
#pragma unroll
            for (int i = 0; i < K; ++i) t8_st<kEStAux>(c.rE, (i < nj && c.live) ? t8_es(c, eoff, i) : kOOB, tt[i]);
            if (idw && c.j == 0 && c.live) t8_st<kEStAux>(c.rE, ((uint32_t)(rc.beg + rc.deg - 1) << 6) + c.eo8, EI);
        }
        // S_col += E_new; slots past the piece add into `dummy` (never read)
        auto sp = [&](int i) { return i < nj ? c.S + (size_t)col[i] * kF8 : c.dummy; };
        // row 2q: half 0's additions after the overlapping wavefronts' row 2q-1
        T8_STAMP(f0);
        T8_ADD(c, 3, q1, f0);
        tp_order(c, 2 * q);
        T8_STAMP(f1);
        T8_ADD(c, 4, f0, f1);
        if (c.h == 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) __hip_atomic_fetch_add(sp(i), tt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        lds_release();
        if ((threadIdx.x & 63) == 0) lds_st(c.p3row + c.wave, 2 * q + 1);
        // row 2q+1: half 1's, after the overlapping wavefronts' row 2q
        T8_STAMP(f2);
        T8_ADD(c, 5, f1, f2);
        tp_order(c, 2 * q + 1);
        T8_STAMP(f3);
        T8_ADD(c, 4, f2, f3);
        if (c.h == 1) {
#pragma unroll
            for (int i = 0; i < K; ++i) __hip_atomic_fetch_add(sp(i), tt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (idw && c.j == 0) {  // identity column: L = ch + (0 + E) (:173-185)
            const double Lj = chI + (0.0 + EI);
            if (c.live) t8_st(c.rL, ((uint32_t)(c.k + r) << 9) + c.lo8, Lj);
            if (!(Lj < 0.0)) atomicOr(c.ib + (r >> 5) * kF8, 1u << (r & 31));
        }
        lds_release();
        if ((threadIdx.x & 63) == 0) lds_st(c.p3row + c.wave, 2 * q + 2);
        T8_STAMP(f4);
        T8_ADD(c, 5, f3, f4);
    };
    if (!tiny_any) {
        // q = P/t (div_nr where exact), then E_new = 2 atanh(clip(q)), or 2q
        // when every quotient of the wavefront is below 2^-27 (exact).
        // Branch-free over all K slots (a padded slot's t = 1.0 gives q = P):
        // per-slot uniform branches made the slots' values merge from many
        // paths (~200 spilled VGPRs).
        const bool dnr = div_nr_ok(c.live ? P : 1.0);
        bool big = false;  // frame-less lanes do not vote
        const double tIx = idw ? tI : 1.0;
        double EI;
        if (dnr) {
#pragma unroll
            for (int i = 0; i < K; ++i) t[i] = div_nr(P, t[i]);
            EI = div_nr(P, tIx);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) t[i] = P / t[i];
            EI = P / tIx;
        }
#pragma unroll
        for (int i = 0; i < K; ++i) big |= !(fabs(t[i]) < kAtanhIdent);
        big |= idw && !(fabs(EI) < kAtanhIdent);
        if (__ballot(big && c.live) == 0ull) {
#pragma unroll
            for (int i = 0; i < K; ++i) t[i] = 2.0 * t[i];
            EI = 2.0 * EI;
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) t[i] = 2.0 * atanh_f(clip_cl(t[i]), c.ltab, ac);
            EI = 2.0 * atanh_f(clip_cl(EI), c.ltab, ac);
        }
        finish(t, EI);
    } else {
        double EI = 0.0;
        // rare: q = in-order product of the others (np.prod(np.delete(...)),
        // :164) for an edge with |t| <= 1e-10 of a tiny row; t parked at row
        // positions (the identity edge at deg-1), every wavefront counts
        const int pos0 = rc.c0 + c.j * rc.CS - rc.beg;
        double *tb = c.Tb + (c.ntiny & 1) * c.tbuf;  // the next rare pair parks in the other buffer
        if (tiny_row) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i < nj) tb[(size_t)(pos0 + i) * kF8] = t[i];
            if (idw && c.j == 0) tb[(size_t)(rc.deg - 1) * kF8] = tI;
        }
        __builtin_amdgcn_s_waitcnt(0);  // scratch stores have reached L2
        c.ntiny += 1;
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c.tseq, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_flag<false>(c.tseq, c.ntiny * kW8);
        auto others = [&](int pos) {
            double qq = 1.0;
            bool fst = true;
            for (int p = 0; p < rc.deg; ++p) {
                if (p == pos) continue;
                const double t2 = ld_l2(tb + (size_t)p * kF8);
                qq = fst ? t2 : qq * t2;
                fst = false;
            }
            return qq;
        };
        // Every live lane's own slots go through E (their E_old is consumed:
        // E is this pass's scratch until E_new lands there), so ONE rolled
        // loop -- one copy of atanh and of the product loop, not K -- turns
        // each into E_new: q = P/t, or for a tiny t of a tiny row the product
        // of the others; then the slots come back into registers.
        const uint32_t eoff = ((uint32_t)(rc.c0 + c.j * rc.CS) << 6) + c.eo8;
#pragma unroll
        for (int i = 0; i < K; ++i) t8_st<kEStAux>(c.rE, (i < nj && c.live) ? t8_es(c, eoff, i) : kOOB, t[i]);
        __builtin_amdgcn_s_waitcnt(0);  // this lane's stores are visible to its own loads
#pragma unroll 1
        for (int i = 0; i < nj; ++i) {
            if (c.live) {
                const double ti = t8_ld(c.rE, t8_es(c, eoff, i));
                const double qv = (tiny_row && !(fabs(ti) > kTiny)) ? others(pos0 + i) : P / ti;
                t8_st<kEStAux>(c.rE, t8_es(c, eoff, i), 2.0 * atanh_f(clip_cl(qv), c.ltab, ac));
            }
        }
        if (idw) {
            const double qv = (!tiny_row || fabs(tI) > kTiny) ? P / tI : others(rc.deg - 1);
            EI = 2.0 * atanh_f(clip_cl(qv), c.ltab, ac);
        }
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int i = 0; i < K; ++i)
            t[i] = t8_ld(c.rE, (i < nj && c.live) ? t8_es(c, eoff, i) : kOOB);  // past the piece: 0 (unused)
        finish(t, EI);
    }
}

// D = 2: body(q) = hop(q), P3(q-1) (staging pair q+1), P1(q+1)
template <int K>
__device__ __forceinline__ void tp_body2(T8Ctx<K> &c, int q, int mp, double (&tc)[K], int yc, double (&to)[K],
                                         int &yo) {
    if (q < mp) tp_hop<K, 2>(c, q, tc, yc);
    T8_STAMP(b0);
    if (q >= 1) tp_p3<K, 2>(c, q - 1, to, tp_stage_issue(c, q + 1));
    T8_STAMP(b1);
    if (q + 1 < mp) yo = tp_p1<K, 2>(c, q + 1, to);
    T8_STAMP(b2);
    T8_ADD(c, 6, b1, b2);
    T8_ADD(c, 7, b0, b1);
}
// One pass over all row pairs (every P3 done on return, before the barrier).
template <int K, int D>
__device__ __forceinline__ void tp_rows(T8Ctx<K> &c) {
    const int mp = (c.m + 1) / 2;  // pairs (an odd m's last pair has an empty second row)
    if (mp <= 0) return;
    static_assert(D == 2, "the pair form runs two pairs in flight (three measured 0.31 vs 0.41: spills)");
    double tA[K], tB[K];
    int yA = 0, yB = 0;
    tp_stage_commit(c, 0, tp_stage_issue(c, 0));
    tp_stage_commit(c, 1, tp_stage_issue(c, 1));
    yA = tp_p1<K, 2>(c, 0, tA);
    for (int q = 0; q <= mp; q += 2) {
        tp_body2(c, q, mp, tA, yA, tB, yB);
        if (q + 1 <= mp) tp_body2(c, q + 1, mp, tB, yB, tA, yA);
    }
}

template <int K, bool LA, bool PAIR, int NS>
__device__ __forceinline__ void t8_setup(T8Ctx<K> &c, unsigned char *lds, const T8Layout &ly, const DevGraph &g,
                                         const DevState &st, int tile, int sub, const int *col_idx,
                                         const int *row_ptr) {
    MathLds &mlds = *(MathLds *)(lds + ly.math);
    int *flags = (int *)(lds + ly.flags);
    const int lane = threadIdx.x & 63;
    c.col_idx = col_idx;
    c.row_ptr = row_ptr;
    c.p3dep = g.p3dep8;
    c.wave = uniform(t8_wave(threadIdx.x >> 6));
    c.j = PAIR ? (lane >> 3) & 3 : lane >> 3;
    c.h = PAIR ? lane >> 5 : 0;
    c.f = lane & 7;
    c.rE = t8_rsrc(st.E + (size_t)tile * g.nnz * kTile + (size_t)sub * g.nnz * kF8,
                   ((size_t)g.nnz + kEPadEdges) * kF8 * sizeof(double));
    c.rL = t8_rsrc(st.L + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));
    c.rC = t8_rsrc(st.ch + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));
    c.eo8 = (uint32_t)c.f * 8u;
    c.lo8 = (uint32_t)(sub * kF8 + c.f) * 8u;
    // rare-row scratch: two buffers of one row per workgroup (of two rows in
    // the pair form: the T pool holds 4 x 8 x 2 x max_row_deg per tile,
    // ldpc_api.cpp workspace)
    c.Tb = st.T + ((size_t)blockIdx.x * (PAIR ? 2 : 1) + c.h) * 2 * g.max_row_deg * kF8 + c.f;
    c.tbuf = (size_t)g.max_row_deg * kF8;
    c.S = (double *)(lds + ly.S) + c.f;
    c.LA = LA ? (double *)(lds + ly.LA) + c.f : nullptr;
    c.dummy = (double *)(lds + ly.dummy) + c.f;
    c.slot = (double *)(lds + ly.slot) + c.f;
    c.ib = (uint32_t *)(lds + ly.ib) + c.f;
    c.cidx = (uint16_t *)(lds + ly.cidx) + c.wave * kQ8 * K;
    c.flag = flags;
    c.ns = NS;
    c.tinyf = flags + NS;
    c.tseq = flags + 2 * NS;
    c.p3row = flags + 2 * NS + 2;
    c.ttab = LdsTanh{mlds.tanh};
    c.ltab = LdsAtanh{mlds.atanh};
    c.m = g.m;
    c.k = g.k;
    c.nnz = g.nnz;
    c.ntiny = 0;
    c.first = false;
    c.fresh = false;
    c.live = true;
    c.ep0 = 0;
#ifdef LDPC_T8_TIMERS
    for (int i = 0; i < T8_NT; ++i) c.tm[i] = 0;
#endif
}

__device__ __forceinline__ int t8_epoch0(int pass, int m) {
    return (int)(((uint32_t)pass * (uint32_t)m) & 0x3ffffffu);
}

// End of a pass: posteriors of the A columns L = ch + S (channel added after
// the sum, :173-185), normalized-LLR count against the previous posterior
// (:210-228), z^1 bits; S cleared.  Thread t owns frame t & 7.
template <bool LA>
__device__ __forceinline__ void t8_vn(const DevGraph &g, double *S, double *LAl, uint32_t *zb, int *cntl,
                                      const int *livel, __amdgpu_buffer_rsrc_t rL, __amdgpu_buffer_rsrc_t rC,
                                      int sub, bool first, bool fresh_any, const int *freshl, int nllr) {
    const int ff = threadIdx.x & 7;
    const uint32_t lo8 = (uint32_t)(sub * kF8 + ff) * 8u;
    const bool live = livel[ff] != 0;
    const bool fr = fresh_any && freshl[ff] != 0;
    int my_cnt = 0;
    for (int e = threadIdx.x; e < g.k * kF8; e += blockDim.x) {
        const int col = e >> 3;
        const double Sj = S[e];
        S[e] = 0.0;
        const double chj = t8_ld(rC, ((uint32_t)col << 9) + lo8);
        const double Lj = chj + Sj;
        if (nllr) {
            double ap;
            if (first || fr)
                ap = chj;
            else if (LA)
                ap = LAl[e];
            else
                ap = t8_ld(rL, ((uint32_t)col << 9) + lo8);
            my_cnt += (fabs(Lj) <= 7.0 && ap * Lj < 0.0) ? 1 : 0;
        }
        if (LA) LAl[e] = Lj;
        if (live) t8_st(rL, ((uint32_t)col << 9) + lo8, Lj);
        if (!(Lj < 0.0)) atomicOr(zb + (col >> 5) * kF8 + ff, 1u << (col & 31));
    }
    if (nllr && my_cnt) atomicAdd(cntl + ff, my_cnt);
}

// syndrome (:191-204): parity of row r = popcount(A_r & (z^1)_A) + (z^1)_{k+r}
__device__ __forceinline__ void t8_syndrome(const DevGraph &g, const uint32_t *zb, const uint32_t *ib, int *bad) {
    const int kw = (g.k + 31) >> 5;
    const int ff = threadIdx.x & 7;
    uint32_t acc = 0u;
    for (int e = threadIdx.x; e < g.m * kF8; e += blockDim.x) {
        const int r = e >> 3;
        const uint32_t *ar = g.a_packed + (size_t)r * kw;
        uint32_t par = ib[(r >> 5) * kF8 + ff] >> (r & 31);
        for (int w = 0; w < kw; ++w) par += __builtin_popcount(ar[w] & zb[w * kF8 + ff]);
        acc |= par & 1u;
    }
    if (acc) atomicOr((uint32_t *)bad + ff, 1u);
}

template <int K, bool LA, int D, bool PAIR = false>
__global__ __launch_bounds__(64 * kW8, 1) void tile8_kernel(DevGraph g, DevState st, int max_iter, int nllr,
                                                            const int *__restrict__ col_idx,
                                                            const int *__restrict__ row_ptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NS = t8_ns(PAIR, D);
    const T8Layout ly = t8_layout(g.k, g.m, K, LA, t8_ring(PAIR, D), NS);
    double *S = (double *)(lds + ly.S);
    double *LAl = LA ? (double *)(lds + ly.LA) : nullptr;
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + kF8;
    int *livel = cntl + kF8;
    int *flags = (int *)(lds + ly.flags);
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x / kQ8, sub = blockIdx.x % kQ8;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(*(MathLds *)(lds + ly.math));
    for (int i = threadIdx.x; i < g.k * kF8; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * kF8; i += blockDim.x) zb[i] = 0u;
    for (int i = threadIdx.x; i < 2 * kF8; i += blockDim.x) bad[i] = 0;
    if (threadIdx.x < 2 * NS) flags[threadIdx.x] = -1;
    if (threadIdx.x >= 2 * NS && threadIdx.x < 2 * NS + 2 + kW8) flags[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < kF8) livel[threadIdx.x] = st.done[tile * kTile + sub * kF8 + threadIdx.x] == 0 ? 1 : 0;
    const __amdgpu_buffer_rsrc_t rC = t8_rsrc(st.ch + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));
    const __amdgpu_buffer_rsrc_t rL = t8_rsrc(st.L + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));
    if constexpr (LA) {  // iteration 0 forms M = ch (:85-90): L_A starts as the channel LLRs
        for (int e = threadIdx.x; e < g.k * kF8; e += blockDim.x)
            LAl[e] = t8_ld(rC, ((uint32_t)(e >> 3) << 9) + (uint32_t)(sub * kF8 + (e & 7)) * 8u);
    }
    __syncthreads();
    if (!st.tile_active[tile]) return;
    {  // a sub-tile with no live frame (a ragged batch's last tile) has nothing to do
        int any = 0;
#pragma unroll
        for (int f = 0; f < kF8; ++f) any |= livel[f];
        if (!any) return;  // block-uniform: LDS after the barrier
    }

    T8Ctx<K> c;
    t8_setup<K, LA, PAIR, NS>(c, lds, ly, g, st, tile, sub, col_idx, row_ptr);
    c.coef_arg = false;  // the static decoder loads them
    c.R = t8_ring(PAIR, D);
    // the identity edge's wavefront: with D = 3 wavefront 0, which otherwise
    // waits longest for the chain; with D = 2 the last one (wavefront 0's
    // body would bound the row period)
    // the identity edge(s) on wavefront 0, first in the chain: the last one's
    // extra P1/P3 work sat on the chain's tail (config 4 static 0.381 -> 0.396,
    // pair form +2.9 %, profiles/r5l_ab, r5m_ab)
    c.idwave = 0;
    const int fr = tile * kTile + sub * kF8 + c.f;  // this lane's frame

    for (int it = 0; it < max_iter; ++it) {
        c.first = it == 0;
        c.live = livel[c.f] != 0;
        c.ep0 = t8_epoch0(it, g.m);
        T8_STAMP(w0);
        if constexpr (PAIR)
            tp_rows<K, D>(c);
        else
            t8_rows<K, LA, D>(c);
        T8_STAMP(w1);
        T8_ADD(c, 8, w0, w1);
        __syncthreads();  // every P3 done: S complete, identity bits set
        if (threadIdx.x < kW8) c.p3row[threadIdx.x] = 0;
        t8_vn<LA>(g, S, LAl, zb, cntl, livel, rL, rC, sub, c.first, false, nullptr, nllr);
        __syncthreads();
        t8_syndrome(g, zb, ib, bad);
        __syncthreads();
        if ((threadIdx.x >> 6) == 0) {  // per-frame exits, as vn_kernel (static schedule)
            bool still = false;
            if (lane < kF8 && livel[lane] != 0) {
                if (nllr) {
                    const int cn = cntl[lane];
                    st.nllr_cnt[fr] = cn;
                    if (st.nllr_hist)
                        st.nllr_hist[(size_t)fr * st.hist_stride + it] = g.k > 0 ? (double)cn / g.k : 0.0;
                }
                if (bad[lane] == 0) {  // syndrome zero: Result.OK at this iteration (:231-241)
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
            if (lane < kF8) {
                livel[lane] = still ? 1 : 0;
                bad[lane] = 0;
                cntl[lane] = 0;
            }
            if (lane == 0) flags[2 * NS + 1] = any != 0ull ? 1 : 0;
        }
        for (int i = threadIdx.x; i < (kw + mw) * kF8; i += blockDim.x) zb[i] = 0u;
        __syncthreads();
        if (!flags[2 * NS + 1]) break;
    }
    count_rare_rows(st, c.tseq, kW8);
#ifdef LDPC_T8_TIMERS
    if ((blockIdx.x == 0 || blockIdx.x == 777) && (threadIdx.x & 63) == 0)
        printf("T8 b=%d w=%d hopw=%llu hop=%llu p3f=%llu p3m=%llu p3o=%llu p3s=%llu p1=%llu pre=%llu rows=%llu\n",
               (int)blockIdx.x, c.wave, (unsigned long long)c.tm[0], (unsigned long long)c.tm[1],
               (unsigned long long)c.tm[2], (unsigned long long)c.tm[3], (unsigned long long)c.tm[4],
               (unsigned long long)c.tm[5], (unsigned long long)c.tm[6], (unsigned long long)c.tm[7],
               (unsigned long long)c.tm[8]);
#endif
}

// Streaming Monte-Carlo on 8-frame sub-tiles (tile_sub.hip's
// tile_sub_stream_kernel at 8 frames per workgroup): every frame slot is at
// its own iteration; after each pass a slot whose frame stopped adds that
// frame's counters (count_kernel's definitions, main.py:130-138) and takes the
// next frame index from one device counter; the whole workgroup generates the
// new frames in place (frame_source.h gen_slots: ch and L = ch, so the frame's
// next pass forms M = L - 0, its iteration 0 -- the `fresh` flag of P1, and
// L_A = ch in LDS for the L_A variant).  Each frame decodes exactly as in the
// static schedule, so the counters are identical.  With handoff > 0 the
// workgroup stops once the supply is out and at most `handoff` frames still
// run anywhere, leaving its slots in the split path's terms (done / iters /
// fresh; E in 8-frame blocks, L, ch and u bits in place) for the
// column-parallel tail (ldpc_api.cpp mc_stream_point).  Reference: the
// per-frame loop of main.py:295-342 over spa_decoder.py:63-280.
template <int K, bool LA, int D, bool PAIR = false>
__global__ __launch_bounds__(64 * kW8, 1) void tile8_stream_kernel(
    DevGraph g, DevState st, int max_iter, int nllr, const int *__restrict__ col_idx,
    const int *__restrict__ row_ptr, AtanhCoef ac, uint64_t seed, int snr_point, double sigma, int64_t frame0,
    int64_t total, unsigned long long *next, unsigned long long *ctr, int64_t handoff) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ long long gidx[kF8];  // refill: slot f's new frame index (< 0: none)
    __shared__ int nref;             // refill: some slot took a frame this pass
    constexpr int NS = t8_ns(PAIR, D);
    const T8Layout ly = t8_layout(g.k, g.m, K, LA, t8_ring(PAIR, D), NS);
    double *S = (double *)(lds + ly.S);
    double *LAl = LA ? (double *)(lds + ly.LA) : nullptr;
    uint32_t *zb = (uint32_t *)(lds + ly.zb);
    uint32_t *ib = (uint32_t *)(lds + ly.ib);
    int *bad = (int *)(lds + ly.lane_i);
    int *cntl = bad + kF8;
    int *livel = cntl + kF8;
    int *itl = livel + kF8;
    int *freshl = itl + kF8;
    int *flags = (int *)(lds + ly.flags);
    const int kw = (g.k + 31) >> 5, mw = (g.m + 31) >> 5;
    const int tile = blockIdx.x / kQ8, sub = blockIdx.x % kQ8;
    if (tile >= st.ntiles) return;  // block-uniform

    fill_math_lds(*(MathLds *)(lds + ly.math));
    for (int i = threadIdx.x; i < g.k * kF8; i += blockDim.x) S[i] = 0.0;
    for (int i = threadIdx.x; i < (kw + mw) * kF8; i += blockDim.x) zb[i] = 0u;
    if (threadIdx.x < 5 * kF8) bad[threadIdx.x] = 0;  // bad, cnt, live, it, fresh
    if (threadIdx.x < 2 * NS) flags[threadIdx.x] = -1;
    if (threadIdx.x >= 2 * NS && threadIdx.x < 2 * NS + 2 + kW8) flags[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    const bool w0 = (threadIdx.x >> 6) == 0;        // hardware wavefront 0 runs the refill and the exits
    const bool slot_lane = threadIdx.x < kF8;       // the lane that owns frame slot f = lane
    bool want = slot_lane;
    const __amdgpu_buffer_rsrc_t rC = t8_rsrc(st.ch + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));
    const __amdgpu_buffer_rsrc_t rL = t8_rsrc(st.L + (size_t)tile * g.n * kTile, (size_t)g.n * kTile * sizeof(double));

    T8Ctx<K> c;
    t8_setup<K, LA, PAIR, NS>(c, lds, ly, g, st, tile, sub, col_idx, row_ptr);
    c.coef_arg = kStreamCoefArg;
    c.ac = ac;
    c.R = t8_ring(PAIR, D);
    c.idwave = 0;  // as tile8_kernel
    const int m = g.m;
    const uint32_t *Ut = st.ubits + (size_t)tile * kw * kTile + sub * kF8 + lane;  // slot lanes only

    for (int pass = 0;; ++pass) {
        __syncthreads();  // the previous pass's exits (or the set-up) are visible
        if (w0) {  // refill: slots without a frame take the next indices
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
                if (slot_lane) gidx[lane] = have ? supply_frame(st, frame0, idx) : -1ll;
                if (want) {
                    livel[lane] = have ? 1 : 0;
                    freshl[lane] = have ? 1 : 0;
                    itl[lane] = 0;
                }
            } else if (slot_lane) {
                gidx[lane] = -1ll;
            }
            const bool gen = __ballot(have) != 0ull;
            want = false;
            const bool go = __ballot(slot_lane && livel[lane] != 0) != 0ull && !stop;
            if (!go && slot_lane) {  // the slots' state, in the split path's terms
                const int fr = tile * kTile + sub * kF8 + lane;
                st.done[fr] = livel[lane] != 0 ? 0 : 1;
                st.iters[fr] = itl[lane];
                st.fresh[fr] = freshl[lane];
                st.refill[fr] = 0;
            }
            if (lane == 0) {
                flags[2 * NS + 1] = go ? 1 : 0;
                nref = go && gen ? 1 : 0;
            }
        }
        __syncthreads();
        if (!flags[2 * NS + 1]) break;  // supply exhausted (or handed off), every slot drained
        if (nref) {  // the new frames, generated by the whole workgroup (u bits staged in zb)
            gen_slots<kF8>(g, st, tile, sub * kF8, gidx, zb, seed, snr_point, sigma);
            if constexpr (LA) {  // a new frame's first pass gathers L = ch
                for (int e = threadIdx.x; e < g.k * kF8; e += blockDim.x)
                    if (gidx[e & 7] >= 0)
                        LAl[e] = t8_ld(rC, ((uint32_t)(e >> 3) << 9) + (uint32_t)(sub * kF8 + (e & 7)) * 8u);
            }
            __syncthreads();
        }
        c.live = livel[c.f] != 0;
        c.fresh = freshl[c.f] != 0;
        c.first = false;
        c.ep0 = t8_epoch0(pass, m);
        if constexpr (PAIR)
            tp_rows<K, D>(c);
        else
            t8_rows<K, LA, D>(c);
        __syncthreads();  // every P3 done: S complete, identity bits set
        if (threadIdx.x < kW8) c.p3row[threadIdx.x] = 0;
        t8_vn<LA>(g, S, LAl, zb, cntl, livel, rL, rC, sub, false, true, freshl, nllr);
        __syncthreads();
        t8_syndrome(g, zb, ib, bad);
        __syncthreads();
        if (w0) {  // per-slot exits and counters (vn_kernel's stream variant)
            unsigned long long cv[7] = {0, 0, 0, 0, 0, 0, 0};
            bool fin = false;
            if (slot_lane && livel[lane] != 0) {
                const int it = itl[lane];
                const bool ok = bad[lane] == 0;  // Result.OK at this iteration (:231-241)
                fin = ok || it == max_iter - 1;  // else DATA_TRANSFER_NOT_OK (:244-253)
                if (fin) {
                    int err = 0;
                    if (!ok)  // main.py:130-138: u vs z^1 of a failed frame
                        for (int w = 0; w < kw; ++w) err += __builtin_popcount(Ut[w * kTile] ^ zb[w * kF8 + lane]);
                    cv[0] = 1;
                    cv[1] = ok ? 0 : 1;
                    cv[2] = (unsigned long long)err;
                    cv[3] = ok ? (unsigned long long)it : 0;
                    cv[4] = ok ? 1 : 0;
                    cv[5] = nllr ? (unsigned long long)cntl[lane] : 0;
                    cv[6] = (unsigned long long)(it + 1);
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
                    const unsigned long long sm = wave_sum(cv[i]);
                    if (lane == 0 && sm) atomicAdd(&ctr[i], sm);
                }
            }
            if (slot_lane) {
                bad[lane] = 0;
                cntl[lane] = 0;
            }
        }
        __syncthreads();  // wave 0 has read zb (error bits) before it is cleared
        for (int i = threadIdx.x; i < (kw + mw) * kF8; i += blockDim.x) zb[i] = 0u;
    }
    count_rare_rows(st, c.tseq, kW8);
}

// Variants: (K, L_A in LDS, pipeline depth D, pair form).  wimax_2304_0.5:
// (5, yes, 3) or the pair form (10, yes, 2 pairs in flight); the r3/4 codes:
// (8, no, 2) -- 8 slots per lane leave no registers for a third row of t.
constexpr int kD5 = 3, kD8 = 2;
template <int K, bool LA, int D, bool PAIR = false>
size_t t8_lds_bytes_k(const DevGraph &g) {
    if (!g.std_form || !g.a_packed || g.k <= 0 || g.n > 65535) return 0;
    const int C = (g.max_row_deg + kW8 - 1) / kW8;
    if ((C + (PAIR ? kPQ : kQ8) - 1) / (PAIR ? kPQ : kQ8) > K) return 0;
    const size_t b = t8_layout(g.k, g.m, K, LA, t8_ring(PAIR, D), t8_ns(PAIR, D)).total;
    return b + 16 <= kLds8Max ? b : 0;  // + the static __shared__ counter(s)
}

// the variant a graph runs: 0 = none, else K * 2 + LA (+ 100: the pair form,
// DevGraph::t8pair, chosen at graph creation)
int t8_variant(const DevGraph &g) {
    if (g.t8pair && t8_lds_bytes_k<10, true, 2, true>(g)) return 121;
    if (t8_lds_bytes_k<5, true, kD5>(g)) return 5 * 2 + 1;
    if (t8_lds_bytes_k<8, false, kD8>(g)) return 8 * 2;
    return 0;
}

}  // namespace

int sub_frames(const DevGraph &g);  // tile_sub.hip

// Whether the 8-frame decoder runs this graph (then its E is laid out in
// 8-frame blocks, DevGraph::ef = 8; read at graph creation).  Default: the
// codes the 16-frame sub-tile decoder cannot hold (the r3/4 codes, k = 1728);
// wimax_2304_0.5 stays on tile_sub_kernel, measured faster.
// LDPC_TILE8=1: every code it can run; 0: none.
bool tile8_applies(const DevGraph &g) {
    const char *e = getenv("LDPC_TILE8");
    const int mode = e ? atoi(e) : -1;
    if (mode == 0 || t8_variant(g) == 0) return false;
    return mode == 1 || sub_frames(g) != 16;
}

bool tile8_pair_fits(const DevGraph &g) { return t8_lds_bytes_k<10, true, 2, true>(g) > 0; }

// rare-row scratch rows per tile of the 8-frame decoder (ldpc_api.cpp sizes
// the T pool: slots >= this x tiles)
int tile8_scratch_per_tile(const DevGraph &g) { return t8_variant(g) >= 100 ? 4 : 2; }

size_t tile8_lds_bytes(const DevGraph &g) {
    switch (t8_variant(g)) {
        case 121: return t8_lds_bytes_k<10, true, 2, true>(g);
        case 11: return t8_lds_bytes_k<5, true, kD5>(g);
        case 16: return t8_lds_bytes_k<8, false, kD8>(g);
        default: return 0;
    }
}

// tile8_stream_kernel's LDS: the static decoder's + gidx[8], nref (static __shared__)
size_t tile8_stream_lds_bytes(const DevGraph &g) {
    const size_t b = tile8_lds_bytes(g);
    return b && b + kF8 * sizeof(long long) + 16 <= kLds8Max ? b : 0;
}

hipError_t launch_tile8_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                               int snr_point, double sigma, int64_t frame0, int64_t total, unsigned long long *next,
                               unsigned long long *ctr, int64_t handoff, hipStream_t s) {
    const size_t lds = tile8_lds_bytes(g);
    if (!tile8_stream_lds_bytes(g) || g.ef != kF8 || !g.a_packed || !st.ubits ||
        st.ntiles * tile8_scratch_per_tile(g) > st.nslots)
        return hipErrorInvalidValue;
    const dim3 grid(st.ntiles * kQ8), block(64 * kW8);
    switch (t8_variant(g)) {
        case 121:
            tile8_stream_kernel<10, true, 2, true><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx,
                                                                         g.row_ptr, kAtanhCoef, seed, snr_point,
                                                                         sigma, frame0, total, next, ctr, handoff);
            break;
        case 11:
            tile8_stream_kernel<5, true, kD5><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx,
                                                                      g.row_ptr, kAtanhCoef, seed, snr_point, sigma,
                                                                      frame0, total, next, ctr, handoff);
            break;
        case 16:
            tile8_stream_kernel<8, false, kD8><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx,
                                                                       g.row_ptr, kAtanhCoef, seed, snr_point, sigma,
                                                                       frame0, total, next, ctr, handoff);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_tile8(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s) {
    const size_t lds = tile8_lds_bytes(g);
    if (!lds || g.ef != kF8 || st.ntiles * tile8_scratch_per_tile(g) > st.nslots) return hipErrorInvalidValue;
    const dim3 grid(st.ntiles * kQ8), block(64 * kW8);
    switch (t8_variant(g)) {
        case 121:
            tile8_kernel<10, true, 2, true><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx,
                                                                  g.row_ptr);
            break;
        case 11:
            tile8_kernel<5, true, kD5><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx, g.row_ptr);
            break;
        case 16:
            tile8_kernel<8, false, kD8><<<grid, block, lds, s>>>(g, st, max_iter, nllr ? 1 : 0, g.col_idx,
                                                                g.row_ptr);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace ldpc
