// ldpc_api.cpp -- the C ABI of libldpc_hip.so (include/ldpc_hip.h).
//
// Host orchestration only: argument checks, device allocation, chunking of a
// batch into frame tiles that fit the workspace, and the per-iteration launch
// sequence (spa_kernels.hip).  Nothing here computes a decode result on the
// CPU: without a GPU every entry point fails with LDPC_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ldpc_internal.h"
#include "spa_device.h"

using ldpc::DevGraph;
using ldpc::DevState;
using ldpc::PhysTile;
using ldpc::kTile;

static thread_local std::string g_last_error;

int ldpc_fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return ldpc_fail(LDPC_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                             __FILE__, __LINE__);                                              \
    } while (0)

struct ldpc_graph {
    int device = 0;
    DevGraph dg{};
    std::vector<int> h_row_ptr, h_col_idx;
    int *d_ints = nullptr;       // one allocation for all index arrays
    uint32_t *d_apack = nullptr;  // bit-packed A (std_form graphs only)
};

struct ldpc_decoder {
    const ldpc_graph *g = nullptr;
    int cap_tiles = 0;
    double *E = nullptr, *T = nullptr, *L = nullptr, *ch = nullptr;
    int *rare = nullptr;  // rare_count[2] + running totals[2] (ldpc_rare_rows_read) + rare_list[cap_tiles*m*4]
    int nslots = 0;
    int *ints = nullptr;  // done, conv, status, iters, nllr_cnt, fresh, refill (cap frames each) + tile_active
    uint32_t *ubits = nullptr;
    // staging for host I/O
    double *llr_stage = nullptr, *post_stage = nullptr;
    uint8_t *z_stage = nullptr;
    // physical mode, HBM-resident state (phys_tile.hip); allocated on first use
    float *pE = nullptr, *pL = nullptr, *pLam = nullptr;
    int64_t pE_cap = 0;  // floats in pE
    int *pbad = nullptr;
    uint8_t *pzb = nullptr;  // [tile][ceil(n/8)][64] hard-decision bytes of the last VN sweep
    uint32_t *pbits = nullptr;
    int *pactive = nullptr;  // [pactive_cap] tiles still running after VN(it)
    int pactive_cap = 0;
    double *hist = nullptr;  // decode's normalized-LLR history [cap][hist_cap], kept between calls
    int hist_cap = 0;        // (main.py's one-frame calls ask for it every time: no hipMalloc per call)
    unsigned long long *counters = nullptr;  // [counters_cap] + 1 frame-index counter (streaming)
    int counters_cap = 0;
    int *cpairs = nullptr;  // streaming tail compaction plan (1 + 2 cap ints), on first use
    uint32_t *tzb = nullptr;  // streaming tail VN: z^1 bits [cap_tiles][ceil(n/32)][64], zero between uses
    int *tcnt = nullptr;      // streaming tail VN: normalized-LLR counts [cap_tiles*64], zero between uses
    int *tbad = nullptr;      // few-frame decode path: row-parity flags [cap_tiles*64], zero between uses
    // streaming supply order (frame_order.hip), grow-only: keys 2 x ord_cap, vals / order ord_cap each
    uint32_t *ord_keys = nullptr;
    int *ord_vals = nullptr, *ord = nullptr;
    int64_t ord_cap = 0;
    void *ord_tmp = nullptr;
    size_t ord_tmp_bytes = 0;
    DevState st{};
    // profiling (ldpc_profile_*)
    bool prof = false;
    struct Span {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Span> spans;
    std::vector<hipEvent_t> pool;
};

namespace {

// scratch slots (max_row_deg x 64 doubles) per tile the tile decoders need:
// two buffers of a row per workgroup (rare rows alternate), four for tile8's
// pair form (two rows per wavefront)
int tile_scratch_rows(const DevGraph &g) { return g.ef == 8 ? ldpc::tile8_scratch_per_tile(g) : 2; }

// Sub-tile decoder's S order (tile_sub.hip sub_p3): wavefront w's P3 of row r
// waits for row r-1's P3 by wavefronts [lo, hi], those whose chunk's extended
// column span (from just past the previous non-empty chunk's last column to
// its own last column; the last non-empty chunk runs to infinity) overlaps
// w's.  Chunking as sub_chunk: C = ceil(deg / 16) edges per wavefront.  An
// empty chunk waits for nothing (lo > hi); after an empty row, every
// wavefront waits for all 16 (whose in-order P3s then cover every row before).
// drop_last: chunk all but each row's last edge (tile8.hip: the identity
// column k + r of an [A | I_m] row is wavefront 0's, outside the chunks).
template <int W = ldpc::kSubWaves>
std::vector<int> sub_p3_deps(int m, const int *row_ptr, const int *col_idx, bool drop_last = false) {
    std::vector<int> dep((size_t)m * W, 1);  // lo 1 > hi 0: no wait
    auto spans = [&](int r, long long lo[W], long long hi[W], bool ne[W]) {
        const int beg = row_ptr[r];
        const int deg = std::max(0, row_ptr[r + 1] - beg - (drop_last ? 1 : 0)), C = (deg + W - 1) / W;
        long long prev = -1;
        int last = -1;
        for (int w = 0; w < W; ++w) {
            const int cnt = std::max(0, std::min(deg - w * C, C));
            ne[w] = cnt > 0;
            if (!ne[w]) continue;
            lo[w] = prev + 1;
            hi[w] = prev = col_idx[beg + w * C + cnt - 1];
            last = w;
        }
        if (last >= 0) hi[last] = LLONG_MAX;
        return last >= 0;
    };
    long long plo[W], phi[W], lo[W], hi[W];
    bool pne[W], ne[W];
    bool prev_any = m > 0 && spans(0, plo, phi, pne);
    for (int r = 1; r < m; ++r) {
        spans(r, lo, hi, ne);
        for (int w = 0; w < W; ++w) {
            if (!ne[w]) continue;
            int vlo = W, vhi = -1;
            for (int v = 0; v < W; ++v)
                if (!prev_any || (pne[v] && plo[v] <= hi[w] && lo[w] <= phi[v])) {
                    vlo = std::min(vlo, v);
                    vhi = std::max(vhi, v);
                }
            dep[(size_t)r * W + w] = vlo > vhi ? 1 : (vlo | vhi << 8);
        }
        std::copy(lo, lo + W, plo);
        std::copy(hi, hi + W, phi);
        std::copy(ne, ne + W, pne);
        prev_any = std::any_of(ne, ne + W, [](bool b) { return b; });
    }
    return dep;
}

int require_gpu() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return ldpc_fail(LDPC_EDEVICE, "no HIP device visible: the SPA decoder runs only on the GPU");
    return LDPC_OK;
}

template <class T>
int dev_alloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return LDPC_OK;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return ldpc_fail(LDPC_ENOMEM, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
    }
    return LDPC_OK;
}

// Message arrays (E: cap x nnz fp64; T: rare-branch scratch) are only needed by
// the parity-mode decoder; physical-mode Monte-Carlo never touches them.
int ensure_messages(ldpc_decoder *d) {
    if (d->E) return LDPC_OK;
    const DevGraph &G = d->g->dg;
    const size_t cap = (size_t)d->cap_tiles * kTile;
    // + kEPadEdges edges of slack: the sub-tile decoder's P1 loads every
    // register slot of a lane group unclamped (tile_sub.hip, sub_p1), up to 63
    // edges past a row's end -- past the last tile's region on its last row
    int rc = dev_alloc(&d->E, cap * (size_t)G.nnz + (size_t)ldpc::kEPadEdges * kTile);
    if (!rc) rc = dev_alloc(&d->T, (size_t)d->nslots * G.max_row_deg * kTile);
    if (rc) {
        (void)hipFree(d->E);
        d->E = nullptr;
    }
    return rc;
}

// IRA generator scratch (parity words) and physical-mode tile state for graph P
// (E32 sized by P's edges: P may differ from the decoder's own graph).
int ensure_pbits(ldpc_decoder *d, const DevGraph &P) {
    if (d->pbits) return LDPC_OK;
    const size_t mw = (size_t)(P.m + 31) / 32, mw32 = (mw + 31) / 32;
    return dev_alloc(&d->pbits, (size_t)d->cap_tiles * (mw + mw32) * kTile);  // pbits + wpar
}

int ensure_phys_tile(ldpc_decoder *d, const DevGraph &P) {
    const size_t cap = (size_t)d->cap_tiles * kTile;
    const int64_t need = (int64_t)(cap * (size_t)P.nnz);
    if (d->pE_cap < need) {
        (void)hipFree(d->pE);
        d->pE = nullptr;
        d->pE_cap = 0;
        if (int rc = dev_alloc(&d->pE, (size_t)need)) return rc;
        d->pE_cap = need;
    }
    if (!d->pL && dev_alloc(&d->pL, cap * (size_t)d->g->dg.n)) return LDPC_ENOMEM;
    if (!d->pLam && dev_alloc(&d->pLam, cap * (size_t)d->g->dg.n)) return LDPC_ENOMEM;
    if (!d->pbad && dev_alloc(&d->pbad, 2 * cap)) return LDPC_ENOMEM;
    if (!d->pzb && dev_alloc(&d->pzb, cap * (size_t)((d->g->dg.n + 7) / 8))) return LDPC_ENOMEM;
    return LDPC_OK;
}

PhysTile phys_tile(ldpc_decoder *d) {
    const DevGraph &G = d->g->dg;
    uint32_t *wpar = d->pbits ? d->pbits + (size_t)d->cap_tiles * ((G.m + 31) / 32) * kTile : nullptr;
    return PhysTile{d->pE, d->pL, d->pLam, d->pbad, d->pbits, wpar, d->cap_tiles * kTile, d->pzb};
}

void state_bind(ldpc_decoder *d, int ntiles, int count) {
    const size_t cap = (size_t)d->cap_tiles * kTile;
    DevState &s = d->st;
    s.E = d->E;
    s.T = d->T;
    s.rare_count = d->rare;
    s.active_count = nullptr;
    s.rare_list = d->rare + 4;
    s.nslots = d->nslots;
    s.L = d->L;
    s.ch = d->ch;
    s.done = d->ints;
    s.conv = d->ints + cap;
    s.status = d->ints + 2 * cap;
    s.iters = d->ints + 3 * cap;
    s.nllr_cnt = d->ints + 4 * cap;
    s.fresh = d->ints + 5 * cap;
    s.refill = d->ints + 6 * cap;
    s.order = nullptr;
    s.tile_active = d->ints + 7 * cap;
    s.ubits = d->ubits;
    s.nllr_hist = nullptr;
    s.hist_stride = 0;
    s.ntiles = ntiles;
    s.count = count;
}

// The graph as one call sees it: LDPC_F_TEST_ZERO switches on the frame
// source's test-only erasures (frame_source.h test_zero_llr) for this call only.
DevGraph call_graph(const ldpc_decoder *d, uint32_t flags) {
    DevGraph G = d->g->dg;
    G.zinj = (flags & LDPC_F_TEST_ZERO) ? 1 : 0;
    return G;
}

hipEvent_t take_event(ldpc_decoder *d) {
    if (!d->pool.empty()) {
        hipEvent_t e = d->pool.back();
        d->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Launch `fn` bracketed by events when profiling is on.
template <class F>
hipError_t timed(ldpc_decoder *d, int kind, hipStream_t s, F &&fn) {
    if (!d->prof) return fn();
    hipEvent_t a = take_event(d), b = take_event(d);
    if (a) (void)hipEventRecord(a, s);
    hipError_t e = fn();
    if (b) (void)hipEventRecord(b, s);
    if (a && b) d->spans.push_back({kind, a, b});
    return e;
}

bool tail_vn_enabled();

// Few tiles of a long-row code: the per-tile vn_kernel (one workgroup per
// tile: ~11 ms a pass) and the sub-tile decoders (one workgroup per 16 or 8
// frames: ~11 / ~6 ms a pass whatever the frame count) are latency-bound there,
// while the split CN + the column-parallel VN (vn_cols_kernel +
// tail_exit_kernel<true>) spread a pass over the chip (~0.3 ms per tile) --
// the drop-in per-frame decode() path (64 slots): one wimax_2304_0.5 frame at
// T=50 in 100 ms instead of 746 ms (tools/probe_decode_latency.py, profiles/
// r3_ab/scols2).  LDPC_SMALL_COLS (read per call): the tile count up to which
// it applies (default: 32 for the 16-frame sub-tile codes, 16 for tile8's
// -- the measured cross-overs; 0 = never).
bool small_batch_cols(const DevGraph &G, int ntiles) {
    if (!G.a_packed || ((G.k + 31) >> 5) > 64 || !tail_vn_enabled()) return false;
    // the 64-frame tile_kernel codes (wimax_576_0.5, BCH): short rows, one launch;
    // beyond the edge path's few frames they stay on tile_kernel
    if (ldpc::tile64_lds_bytes(G) > 0) return false;
    const char *e = getenv("LDPC_SMALL_COLS");
    const int lim = e ? atoi(e) : (G.ef == 8 ? 16 : 32);
    if (ntiles > lim) return false;
    return !ldpc::use_tile(G) || ldpc::sub_frames(G) == 16 || G.ef == 8;
}

// Few frames: the lanes of a wavefront take a row's / column's edges instead
// of frames (edge_kernels.hip), so a pass's loads are all in flight at once --
// main.py's one-frame decode() calls: one wimax_2304_0.5 frame at T=50 in
// 5.1 ms instead of 102 ms (4.3 ms since), 8 frames in 20 ms (a frame costs ~2 ms more;
// profiles/r3g_edge).  LDPC_EDGE_FRAMES (read per call): the batch size up to
// which it applies (default 32 for the 2304 codes, below the frame-per-lane
// path's ~100 ms; 4 for the codes of the 64-frame tile_kernel, whose one
// launch takes 7.9 ms for wimax_576_0.5 against 2.9 ms + ~1.1 ms per frame;
// 0 = never; LDPC_SMALL_COLS=0, which keeps every small-batch path away, too).
bool small_batch_edge(const DevGraph &G, int count) {
    const char *c = getenv("LDPC_SMALL_COLS");
    if (c && atoi(c) == 0) return false;
    const char *e = getenv("LDPC_EDGE_FRAMES");
    const int lim = e ? atoi(e) : (ldpc::tile64_lds_bytes(G) > 0 ? 4 : 32);
    return count <= lim && G.max_row_deg <= ldpc::edge_max_deg() && G.max_col_deg <= ldpc::edge_max_deg();
}

// the column-parallel VN's per-tile buffers (zero between passes).  Each
// buffer is allocated under its own null check, so a failed allocation leaves
// the others consistent and a later call retries only what is missing.
int ensure_tail_bufs(ldpc_decoder *d, hipStream_t s) {
    const DevGraph &G = d->g->dg;
    const int cap = d->cap_tiles * kTile;
    const size_t nzb = (size_t)d->cap_tiles * ((G.n + 31) / 32) * kTile;
    if (!d->tzb)
        if (int rc = dev_alloc(&d->tzb, nzb)) return rc;
    if (!d->tcnt)
        if (int rc = dev_alloc(&d->tcnt, (size_t)cap)) return rc;
    if (!d->tbad)
        if (int rc = dev_alloc(&d->tbad, (size_t)cap)) return rc;
    // tail_exit_kernel leaves them zero, but a call that stopped early (an
    // error return) may not have: cleared per call, never trusted
    if (hipMemsetAsync(d->tzb, 0, nzb * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(d->tcnt, 0, (size_t)cap * sizeof(int), s) != hipSuccess ||
        hipMemsetAsync(d->tbad, 0, (size_t)cap * sizeof(int), s) != hipSuccess)
        return ldpc_fail(LDPC_EDEVICE, "tail buffers: memset failed");
    return LDPC_OK;
}

// Up to max_iter CN/VN sweeps.  With poll (callers that synchronise anyway),
// the host reads how many tiles are still running after VN(it) for it < 4 and
// every 4th iteration after, and stops once none is: launches over finished
// tiles cost ~0.3 ms each (a grid of early-exiting workgroups).  Which path
// runs is decided first (few-frame edge path, small-batch column-parallel VN,
// the tile-resident decoder, or the split CN/VN launches); an allocation or
// HIP failure is returned as an LDPC_E* code, never turned into another path.
int run_iterations(ldpc_decoder *d, const DevGraph &G, const DevState &st_in, int max_iter, bool nllr,
                   hipStream_t s, bool poll, bool split) {
    DevState st = st_in;
    // the edge path applies to every [A | I] code with k <= 2048 (the 64-frame
    // tile codes too: one wimax_576_0.5 frame, profiles/r3g_edge)
    const bool cols_ok = G.a_packed && ((G.k + 31) >> 5) <= 64 && tail_vn_enabled();
    const bool edge = cols_ok && small_batch_edge(G, st.count);
    const bool cols = edge || (cols_ok && small_batch_cols(G, st.ntiles));
    if (cols)
        if (int rc = ensure_tail_bufs(d, s)) return rc;
    auto hip = [](hipError_t e) {
        return e == hipSuccess ? LDPC_OK
                               : ldpc_fail(LDPC_EDEVICE, "decode iterations: %s", hipGetErrorString(e));
    };
    if (!split && !cols && ldpc::use_tile(G) && st.ntiles * tile_scratch_rows(G) <= st.nslots)  // one launch: every tile to its own exit
        return hip(timed(d, LDPC_K_TILE, s, [&] { return ldpc::launch_tile(G, st, max_iter, nllr, s); }));
    // cn_rare_kernel clears the OTHER parity's count for the next CN; the one
    // the last iteration used (or an early stop left) is cleared here
    hipError_t e = hipMemsetAsync(st.rare_count, 0, sizeof(int) * 2, s);
    if (e) return hip(e);
    if (poll) {
        if (d->pactive_cap < max_iter) {
            (void)hipFree(d->pactive);
            d->pactive = nullptr;
            d->pactive_cap = 0;
            if (int rc = dev_alloc(&d->pactive, (size_t)max_iter)) return rc;
            d->pactive_cap = max_iter;
        }
        if ((e = hipMemsetAsync(d->pactive, 0, sizeof(int) * max_iter, s))) return hip(e);
        st.active_count = d->pactive;
    }
    for (int it = 0; it < max_iter && e == hipSuccess; ++it) {
        if (edge) {  // the rare rows are handled inside cn_edge_kernel
            e = timed(d, LDPC_K_CN_EDGE, s, [&] { return ldpc::launch_cn_edge(G, st, it, s); });
        } else {
            e = timed(d, LDPC_K_CN, s, [&] { return ldpc::launch_cn(G, st, it, s); });
            if (e == hipSuccess) e = ldpc::launch_cn_rare(G, st, it, s);
        }
        if (e == hipSuccess) {
            const bool last = it + 1 == max_iter;
            if (edge)
                e = timed(d, LDPC_K_VN_EDGE, s, [&] {
                    return ldpc::launch_vn_edge_decode(G, st, it, last, nllr, d->tzb, d->tcnt, d->tbad, s);
                });
            else if (cols)
                e = timed(d, LDPC_K_VN_COLS, s, [&] {
                    return ldpc::launch_vn_cols_decode(G, st, it, last, nllr, d->tzb, d->tcnt, s);
                });
            else
                e = timed(d, LDPC_K_VN, s, [&] { return ldpc::launch_vn(G, st, it, max_iter, nllr, s); });
        }
        if (e == hipSuccess && poll && it + 1 < max_iter && (it < 4 || (it + 1) % 4 == 0)) {
            int running = 0;
            e = hipMemcpyAsync(&running, d->pactive + it, sizeof(int), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess && running == 0) break;
        }
    }
    return hip(e);
}

// cn_rare_kernel runs 1024 blocks x 4 wavefronts; one scratch slot each.
int scratch_slots() { return 4096; }


size_t workspace_bytes(const DevGraph &g, int cap_tiles) {
    const size_t cap = (size_t)cap_tiles * kTile;
    const size_t kw = (size_t)((g.k + 31) / 32);
    size_t b = 0;
    b += cap * (size_t)g.nnz * 8;                                   // E
    const size_t slots = ldpc::use_tile(g) ? std::max(scratch_slots(), cap_tiles * tile_scratch_rows(g)) : scratch_slots();
    b += slots * g.max_row_deg * kTile * 8;  // T pool
    b += 4 * (4 + (size_t)cap_tiles * g.m * 4);                           // rare counts + list
    b += 2 * cap * (size_t)g.n * 8;    // L, ch
    b += (7 * cap + cap_tiles) * 4;    // per-frame ints + tile flags
    b += cap * kw * 4;                 // ubits
    b += 2 * cap * (size_t)g.n * 8;    // llr/post staging
    b += cap * (size_t)g.n;            // z staging
    b += cap * ((size_t)(g.n + 31) / 32) * 4 + 2 * cap * 4;  // column-parallel VN / few-frame buffers (tzb, tcnt, tbad)
    // not included: the normalized-LLR history of decode() calls that ask for
    // it (cap x max_iter doubles, allocated on first use, grow-only) and the
    // Monte-Carlo counters (7 int64 per SNR point)
    return b;
}

}  // namespace

extern "C" {

const char *ldpc_last_error(void) { return g_last_error.c_str(); }
int ldpc_abi_version(void) { return LDPC_ABI_VERSION; }

int ldpc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ------------------------------------------------------------------ graph
int ldpc_graph_create(int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx, int32_t device,
                      ldpc_graph **out) {
    if (!out) return ldpc_fail(LDPC_EINVAL, "ldpc_graph_create: out is NULL");
    *out = nullptr;
    if (m <= 0 || n <= 0 || m > n || !row_ptr || !col_idx)
        return ldpc_fail(LDPC_EINVAL, "ldpc_graph_create: bad shape m=%d n=%d", m, n);
    if (row_ptr[0] != 0) return ldpc_fail(LDPC_EINVAL, "ldpc_graph_create: row_ptr[0] != 0");
    const int64_t nnz = row_ptr[m];
    // within-tile offsets are 32-bit: e*64 must fit
    if (nnz <= 0 || nnz > (int64_t)(INT32_MAX / kTile) || (int64_t)n > (int64_t)(INT32_MAX / kTile))
        return ldpc_fail(LDPC_ERANGE, "ldpc_graph_create: nnz=%lld outside 32-bit tile indexing", (long long)nnz);
    int max_row = 0;
    for (int r = 0; r < m; ++r) {
        const int b = row_ptr[r], e = row_ptr[r + 1];
        if (e < b) return ldpc_fail(LDPC_EINVAL, "ldpc_graph_create: row_ptr not monotone at %d", r);
        max_row = std::max(max_row, e - b);
        for (int i = b; i < e; ++i) {
            if (col_idx[i] < 0 || col_idx[i] >= n)
                return ldpc_fail(LDPC_EINVAL, "ldpc_graph_create: column %d out of range", col_idx[i]);
            if (i > b && col_idx[i] <= col_idx[i - 1])
                return ldpc_fail(LDPC_EINVAL,
                                 "ldpc_graph_create: row %d columns not strictly ascending "
                                 "(the reference's check_to_var order is required)",
                                 r);
        }
    }
    if (int rc = require_gpu()) return rc;
    auto *g = new ldpc_graph;
    g->h_row_ptr.assign(row_ptr, row_ptr + m + 1);
    g->h_col_idx.assign(col_idx, col_idx + nnz);
    // CSC view with rows ascending (var_to_check order; also the order scipy's
    // E.tocsc() sums a column in, spa_decoder.py:177-182)
    std::vector<int> csc_ptr(n + 1, 0), csc_edge(nnz), csc_row(nnz);
    for (int64_t e = 0; e < nnz; ++e) csc_ptr[col_idx[e] + 1]++;
    for (int j = 0; j < n; ++j) csc_ptr[j + 1] += csc_ptr[j];
    std::vector<int> fill(csc_ptr.begin(), csc_ptr.end() - 1);
    int max_col = 0;
    for (int j = 0; j < n; ++j) max_col = std::max(max_col, csc_ptr[j + 1] - csc_ptr[j]);
    for (int r = 0; r < m; ++r)
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
            const int p = fill[col_idx[e]]++;
            csc_edge[p] = e;
            csc_row[p] = r;
        }
    const int k = n - m;
    // standard form check: row r's only column >= k is k+r (encoder needs it)
    int std_form = 1;
    for (int r = 0; r < m && std_form; ++r) {
        int hits = 0;
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e)
            if (col_idx[e] >= k) hits += (col_idx[e] == k + r) ? 1 : 100;
        std_form = hits == 1;
    }
    // IRA form: the parity columns are exactly the staircase p_r in rows r, r+1
    int ira = k > 0 && !std_form;
    for (int r = 0; r < m && ira; ++r) {
        int hits = 0;
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e)
            if (col_idx[e] >= k) hits += (col_idx[e] == k + r || (r > 0 && col_idx[e] == k + r - 1)) ? 1 : 100;
        ira = hits == (r > 0 ? 2 : 1);
    }
    g->device = device;
    DeviceGuard dg(device);
    if (device < 0) (void)hipGetDevice(&g->device);
    const std::vector<int> p3dep = sub_p3_deps(m, row_ptr, col_idx);
    const std::vector<int> p3dep8 = sub_p3_deps(m, row_ptr, col_idx, true);
    const size_t nints = (size_t)(m + 1) + nnz + (size_t)(n + 1) + 2 * (size_t)nnz + p3dep.size() + p3dep8.size();
    if (int rc = dev_alloc(&g->d_ints, nints)) {
        delete g;
        return rc;
    }
    int *p = g->d_ints;
    DevGraph &G = g->dg;
    G.m = m;
    G.n = n;
    G.k = k;
    G.nnz = (int)nnz;
    G.max_row_deg = max_row;
    G.max_col_deg = max_col;
    G.std_form = std_form;
    G.ira = ira;
    G.ef = kTile;
    {
        int odd = 0;
        for (int r = 0; r < m; ++r) odd += (row_ptr[r + 1] - row_ptr[r]) & 1;
        G.lpt_weak_id = std_form && m > 0 && 2 * odd <= m;
    }
    G.row_ptr = p;
    p += m + 1;
    G.col_idx = p;
    p += nnz;
    G.csc_ptr = p;
    p += n + 1;
    G.csc_edge = p;
    p += nnz;
    G.csc_row = p;
    p += nnz;
    G.p3dep = p;
    p += p3dep.size();
    G.p3dep8 = p;
    p += p3dep8.size();
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMemcpy((void *)G.row_ptr, row_ptr, sizeof(int) * (m + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy((void *)G.col_idx, col_idx, sizeof(int) * nnz, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy((void *)G.csc_ptr, csc_ptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy((void *)G.csc_edge, csc_edge.data(), sizeof(int) * nnz, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy((void *)G.csc_row, csc_row.data(), sizeof(int) * nnz, hipMemcpyHostToDevice);
    if (e == hipSuccess && m > 0)
        e = hipMemcpy((void *)G.p3dep, p3dep.data(), sizeof(int) * p3dep.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && m > 0)
        e = hipMemcpy((void *)G.p3dep8, p3dep8.data(), sizeof(int) * p3dep8.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && std_form && k > 0) {  // encoder table: A bit-packed per row
        const size_t kw = (size_t)(k + 31) / 32;
        std::vector<uint32_t> ap((size_t)m * kw, 0u);
        for (int r = 0; r < m; ++r)
            for (int i = row_ptr[r]; i < row_ptr[r + 1]; ++i)
                if (col_idx[i] < k) ap[(size_t)r * kw + (col_idx[i] >> 5)] |= 1u << (col_idx[i] & 31);
        if (dev_alloc(&g->d_apack, ap.size())) e = hipErrorOutOfMemory;
        if (e == hipSuccess)
            e = hipMemcpy(g->d_apack, ap.data(), sizeof(uint32_t) * ap.size(), hipMemcpyHostToDevice);
        G.a_packed = g->d_apack;
    }
    // the WiMAX 2304 codes run the 8-frame sub-tile decoder: E in 8-frame blocks
    if (e == hipSuccess && !ldpc::tile64_lds_bytes(G) && ldpc::tile8_applies(G)) G.ef = 8;
    // its pair form (two rows per wavefront): LDPC_T8_PAIR=1 (A/B)
    if (G.ef == 8 && ldpc::tile8_pair_fits(G)) {
        const char *ep = getenv("LDPC_T8_PAIR");
        G.t8pair = ep && atoi(ep) != 0 ? 1 : 0;
    }
    if (e != hipSuccess) {
        (void)hipFree(g->d_ints);
        (void)hipFree(g->d_apack);
        delete g;
        return ldpc_fail(LDPC_EDEVICE, "ldpc_graph_create: upload failed: %s", hipGetErrorString(e));
    }
    *out = g;
    return LDPC_OK;
}

int ldpc_graph_destroy(ldpc_graph *g) {
    if (!g) return LDPC_OK;
    DeviceGuard dg(g->device);
    (void)hipFree(g->d_ints);
    (void)hipFree(g->d_apack);
    delete g;
    return LDPC_OK;
}

const char *ldpc_cn_kernel_name(const ldpc_graph *g) {
    if (!g) return "";
    return ldpc::use_cn_row(g->dg) ? "cn_row_kernel" : "cn_kernel";
}

const char *ldpc_tile_kernel_name(const ldpc_graph *g) {
    if (!g || !ldpc::use_tile(g->dg)) return "";
    return ldpc::tile_kernel_name(g->dg);
}

int64_t ldpc_tile_lds_bytes(const ldpc_graph *g) {
    if (!g) return 0;
    return ldpc::use_tile(g->dg) ? (int64_t)ldpc::tile_lds_bytes(g->dg) : 0;
}

namespace {
bool phys_use_lds(const DevGraph &P, uint32_t flags);
}

const char *ldpc_phys_kernel_name(const ldpc_graph *g, uint32_t flags) {
    if (!g) return "";
    if (!phys_use_lds(g->dg, flags)) return "phys_cn_tile_kernel";
    return ldpc::phys_block_threads(g->dg) > 256 ? "phys_reg_kernel" : "phys_kernel";
}

int ldpc_graph_info(const ldpc_graph *g, int32_t *m, int32_t *n, int64_t *nnz, int32_t *max_row_deg,
                    int32_t *max_col_deg) {
    if (!g) return ldpc_fail(LDPC_EINVAL, "ldpc_graph_info: NULL graph");
    if (m) *m = g->dg.m;
    if (n) *n = g->dg.n;
    if (nnz) *nnz = g->dg.nnz;
    if (max_row_deg) *max_row_deg = g->dg.max_row_deg;
    if (max_col_deg) *max_col_deg = g->dg.max_col_deg;
    return LDPC_OK;
}

// ---------------------------------------------------------------- decoder
int64_t ldpc_decoder_bytes(const ldpc_graph *g, int32_t max_frames) {
    if (!g || max_frames <= 0) return -1;
    const int tiles = (max_frames + kTile - 1) / kTile;
    return (int64_t)workspace_bytes(g->dg, tiles);
}

int ldpc_decoder_create(const ldpc_graph *g, int32_t max_frames, ldpc_decoder **out) {
    if (!out) return ldpc_fail(LDPC_EINVAL, "ldpc_decoder_create: out is NULL");
    *out = nullptr;
    if (!g || max_frames <= 0) return ldpc_fail(LDPC_EINVAL, "ldpc_decoder_create: bad arguments");
    DeviceGuard dg(g->device);
    auto *d = new ldpc_decoder;
    d->g = g;
    d->cap_tiles = (max_frames + kTile - 1) / kTile;
    const size_t cap = (size_t)d->cap_tiles * kTile;
    const DevGraph &G = g->dg;
    const size_t kw = (size_t)((G.k + 31) / 32);
    int rc = LDPC_OK;
    d->nslots = scratch_slots();  // E and T are allocated on first parity-mode use
    if (ldpc::use_tile(G))  // one scratch row per tile workgroup (two for tile8's pair form)
        d->nslots = std::max(d->nslots, d->cap_tiles * tile_scratch_rows(G));
    // rare list: one entry per (tile, row), or per 16-frame sub-tile of it (cn_sub_kernel);
    // entries pack tile * m + row into 28 bits (spa_device.h rare_code)
    if ((int64_t)d->cap_tiles * G.m >= (int64_t)1 << 28) {
        delete d;
        return ldpc_fail(LDPC_ERANGE, "ldpc_decoder_create: %d frames x %d rows exceed the rare-row list", max_frames,
                         G.m);
    }
    if (!rc) rc = dev_alloc(&d->rare, 4 + (size_t)d->cap_tiles * G.m * 4);
    if (!rc && hipMemset(d->rare, 0, sizeof(int) * 4) != hipSuccess)
        rc = ldpc_fail(LDPC_EDEVICE, "ldpc_decoder_create: memset failed");
    if (!rc) rc = dev_alloc(&d->L, cap * (size_t)G.n);
    if (!rc) rc = dev_alloc(&d->ch, cap * (size_t)G.n);
    if (!rc) rc = dev_alloc(&d->ints, 7 * cap + (size_t)d->cap_tiles);
    if (!rc) rc = dev_alloc(&d->ubits, std::max<size_t>(cap * kw, 1));
    if (!rc) rc = dev_alloc(&d->llr_stage, cap * (size_t)G.n);
    if (!rc) rc = dev_alloc(&d->post_stage, cap * (size_t)G.n);
    if (!rc) rc = dev_alloc(&d->z_stage, cap * (size_t)G.n);
    if (rc) {
        ldpc_decoder_destroy(d);
        return rc;
    }
    *out = d;
    return LDPC_OK;
}

int ldpc_decoder_destroy(ldpc_decoder *d) {
    if (!d) return LDPC_OK;
    DeviceGuard dg(d->g ? d->g->device : -1);
    (void)hipFree(d->E);
    (void)hipFree(d->T);
    (void)hipFree(d->rare);
    (void)hipFree(d->cpairs);
    (void)hipFree(d->tzb);
    (void)hipFree(d->tcnt);
    (void)hipFree(d->tbad);
    (void)hipFree(d->ord_keys);
    (void)hipFree(d->ord_vals);
    (void)hipFree(d->ord);
    (void)hipFree(d->ord_tmp);
    (void)hipFree(d->hist);
    (void)hipFree(d->L);
    (void)hipFree(d->ch);
    (void)hipFree(d->ints);
    (void)hipFree(d->ubits);
    (void)hipFree(d->llr_stage);
    (void)hipFree(d->post_stage);
    (void)hipFree(d->z_stage);
    (void)hipFree(d->counters);
    (void)hipFree(d->pE);
    (void)hipFree(d->pL);
    (void)hipFree(d->pLam);
    (void)hipFree(d->pbad);
    (void)hipFree(d->pzb);
    (void)hipFree(d->pbits);
    (void)hipFree(d->pactive);
    for (auto &sp : d->spans) {
        (void)hipEventDestroy(sp.a);
        (void)hipEventDestroy(sp.b);
    }
    for (auto e : d->pool) (void)hipEventDestroy(e);
    delete d;
    return LDPC_OK;
}

int32_t ldpc_decoder_capacity(const ldpc_decoder *d) { return d ? d->cap_tiles * kTile : 0; }

// ----------------------------------------------------------------- decode
int ldpc_decode_f64(ldpc_decoder *d, int32_t batch, const double *llr, int32_t max_iter, uint32_t flags,
                    uint8_t *z_out, int32_t *conv_out, int32_t *status_out, double *post_out, double *nllr_out,
                    double *nllr_hist, int32_t *iters_out, double *msg_out, void *stream) {
    if (!d) return ldpc_fail(LDPC_EINVAL, "ldpc_decode_f64: NULL decoder");
    if (batch < 0) return ldpc_fail(LDPC_EINVAL, "ldpc_decode_f64: batch < 0");
    if (max_iter < 1)
        return ldpc_fail(LDPC_EINVAL,
                         "ldpc_decode_f64: max_iter=%d; must be >= 1 (the reference loops until the "
                         "syndrome clears for T<1, spa_decoder.py:104)",
                         max_iter);
    if (batch == 0) return LDPC_OK;
    if (!llr) return ldpc_fail(LDPC_EINVAL, "ldpc_decode_f64: llr is NULL");
    const bool dev_ptrs = flags & LDPC_F_DEVICE_PTRS;
    const bool nllr = flags & LDPC_F_NLLR;
    if (dev_ptrs && msg_out) return ldpc_fail(LDPC_EINVAL, "ldpc_decode_f64: msg_out is host-only");
    DeviceGuard dg(d->g->device);
    if (int rc0 = ensure_messages(d)) return rc0;
    hipStream_t s = (hipStream_t)stream;
    const DevGraph &G = d->g->dg;
    const int n = G.n;
    const int cap = d->cap_tiles * kTile;

    double *d_hist = nullptr;
    double *d_msgs = nullptr;
    std::vector<int> h_ints;
    std::vector<double> h_dbl;
    int rc = LDPC_OK;
    if (nllr_hist) {
        if (d->hist_cap < max_iter) {  // grow-only, reused by later calls
            (void)hipFree(d->hist);
            d->hist = nullptr;
            d->hist_cap = 0;
            if ((rc = dev_alloc(&d->hist, (size_t)cap * max_iter))) return rc;
            d->hist_cap = max_iter;
        }
        d_hist = d->hist;
    }
    if (msg_out) {
        if ((rc = dev_alloc(&d_msgs, (size_t)cap * G.nnz))) return rc;
    }
    auto fail_dev = [&](hipError_t e, const char *what) {
        (void)hipFree(d_msgs);
        return ldpc_fail(LDPC_EDEVICE, "ldpc_decode_f64: %s: %s", what, hipGetErrorString(e));
    };
    hipError_t e = hipSuccess;
    for (int start = 0; start < batch; start += cap) {
        const int cnt = std::min(cap, batch - start);
        const int ntiles = (cnt + kTile - 1) / kTile;
        state_bind(d, ntiles, cnt);
        DevState st = d->st;
        if (d_hist) {
            st.nllr_hist = d_hist;
            st.hist_stride = max_iter;
            if ((e = hipMemsetD8Async((hipDeviceptr_t)d_hist, 0xFF, sizeof(double) * (size_t)cnt * max_iter, s)))
                return fail_dev(e, "memset");
        }
        const double *src = llr + (size_t)start * n;
        if (!dev_ptrs) {
            if ((e = hipMemcpyAsync(d->llr_stage, src, sizeof(double) * (size_t)cnt * n, hipMemcpyHostToDevice, s)))
                return fail_dev(e, "llr upload");
            src = d->llr_stage;
        }
        if ((e = ldpc::launch_reset(G, st, s))) return fail_dev(e, "reset");
        if ((e = ldpc::launch_load_llr(G, st, src, s))) return fail_dev(e, "load");
        if (int rc1 = run_iterations(d, G, st, max_iter, nllr, s, !dev_ptrs, flags & LDPC_F_SPLIT)) {
            (void)hipFree(d_msgs);
            return rc1;
        }
        uint8_t *zdst = dev_ptrs ? (z_out ? z_out + (size_t)start * n : nullptr) : d->z_stage;
        double *pdst = dev_ptrs ? (post_out ? post_out + (size_t)start * n : nullptr) : (post_out ? d->post_stage : nullptr);
        if (zdst || pdst) {
            uint8_t *zz = zdst ? zdst : d->z_stage;
            if ((e = ldpc::launch_finalize(G, st, zz, pdst, s))) return fail_dev(e, "finalize");
        }
        if (d_msgs && (e = ldpc::launch_export_msgs(G, st, d_msgs, s))) return fail_dev(e, "export");
        // per-frame scalars
        const size_t capz = (size_t)d->cap_tiles * kTile;
        auto copy_ints = [&](int32_t *dst, const int *srcp) -> hipError_t {
            if (!dst) return hipSuccess;
            return hipMemcpyAsync(dst + start, srcp, sizeof(int) * cnt,
                                  dev_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s);
        };
        if ((e = copy_ints(conv_out, st.conv))) return fail_dev(e, "conv copy");
        if ((e = copy_ints(status_out, st.status))) return fail_dev(e, "status copy");
        if ((e = copy_ints(iters_out, st.iters))) return fail_dev(e, "iters copy");
        (void)capz;
        if (!dev_ptrs) {
            if (z_out && (e = hipMemcpyAsync(z_out + (size_t)start * n, d->z_stage, (size_t)cnt * n,
                                             hipMemcpyDeviceToHost, s)))
                return fail_dev(e, "z copy");
            if (post_out && (e = hipMemcpyAsync(post_out + (size_t)start * n, d->post_stage,
                                                sizeof(double) * (size_t)cnt * n, hipMemcpyDeviceToHost, s)))
                return fail_dev(e, "post copy");
            if (msg_out && (e = hipMemcpyAsync(msg_out + (size_t)start * G.nnz, d_msgs,
                                               sizeof(double) * (size_t)cnt * G.nnz, hipMemcpyDeviceToHost, s)))
                return fail_dev(e, "msg copy");
            if (nllr_hist && (e = hipMemcpyAsync(nllr_hist + (size_t)start * max_iter, d_hist,
                                                 sizeof(double) * (size_t)cnt * max_iter, hipMemcpyDeviceToHost, s)))
                return fail_dev(e, "hist copy");
            if (nllr_out) {
                h_ints.resize(cnt);
                if ((e = hipMemcpyAsync(h_ints.data(), st.nllr_cnt, sizeof(int) * cnt, hipMemcpyDeviceToHost, s)))
                    return fail_dev(e, "nllr copy");
                if ((e = hipStreamSynchronize(s))) return fail_dev(e, "sync");
                for (int i = 0; i < cnt; ++i)
                    nllr_out[start + i] = nllr ? (G.k > 0 ? (double)h_ints[i] / G.k : 0.0) : 0.0;
            }
            // the staging buffers are reused by the next chunk
            if ((e = hipStreamSynchronize(s))) return fail_dev(e, "sync");
        } else if (nllr_out || nllr_hist) {
            if (nllr_hist && (e = hipMemcpyAsync(nllr_hist + (size_t)start * max_iter, d_hist,
                                                 sizeof(double) * (size_t)cnt * max_iter, hipMemcpyDeviceToDevice, s)))
                return fail_dev(e, "hist copy");
            if (nllr_out) {  // device path: convert counts on the host side of the stream
                h_ints.resize(cnt);
                h_dbl.resize(cnt);
                if ((e = hipMemcpyAsync(h_ints.data(), st.nllr_cnt, sizeof(int) * cnt, hipMemcpyDeviceToHost, s)))
                    return fail_dev(e, "nllr copy");
                if ((e = hipStreamSynchronize(s))) return fail_dev(e, "sync");
                for (int i = 0; i < cnt; ++i) h_dbl[i] = nllr ? (G.k > 0 ? (double)h_ints[i] / G.k : 0.0) : 0.0;
                if ((e = hipMemcpy(nllr_out + start, h_dbl.data(), sizeof(double) * cnt, hipMemcpyHostToDevice)))
                    return fail_dev(e, "nllr upload");
            }
        }
    }
    if (d_hist || d_msgs) {
        if ((e = hipStreamSynchronize(s))) return fail_dev(e, "sync");
    }
    (void)hipFree(d_msgs);
    if ((e = hipGetLastError())) return ldpc_fail(LDPC_EDEVICE, "ldpc_decode_f64: %s", hipGetErrorString(e));
    return LDPC_OK;
}

// ------------------------------------------------------- Monte-Carlo path
int ldpc_generate_frames(ldpc_decoder *d, uint64_t seed, int32_t snr_point, double sigma, int64_t frame0,
                         int32_t count, uint32_t flags, uint8_t *u_out, double *llr_out, void *stream) {
    if (!d) return ldpc_fail(LDPC_EINVAL, "ldpc_generate_frames: NULL decoder");
    const DevGraph G = call_graph(d, flags);
    if (!G.std_form && !G.ira)
        return ldpc_fail(LDPC_EINVAL, "ldpc_generate_frames: graph is neither [A | I_m] nor IRA [H_info | staircase]");
    if (count < 0 || count > d->cap_tiles * kTile || snr_point < 0 || frame0 < 0 || !(sigma > 0.0))
        return ldpc_fail(LDPC_EINVAL, "ldpc_generate_frames: bad arguments (count=%d cap=%d)", count,
                         d->cap_tiles * kTile);
    if (count == 0) return LDPC_OK;
    DeviceGuard dg(d->g->device);
    hipStream_t s = (hipStream_t)stream;
    const bool dev_ptrs = flags & LDPC_F_DEVICE_PTRS;
    state_bind(d, (count + kTile - 1) / kTile, count);
    uint8_t *u_dev = nullptr;
    double *l_dev = nullptr;
    int rc = LDPC_OK;
    if (!dev_ptrs) {
        if (u_out && (rc = dev_alloc(&u_dev, (size_t)count * G.k))) return rc;
        l_dev = llr_out ? d->llr_stage : nullptr;
    } else {
        u_dev = u_out;
        l_dev = llr_out;
    }
    if ((rc = ensure_pbits(d, G))) {
        (void)hipFree(dev_ptrs ? nullptr : u_dev);
        return rc;
    }
    HIP_TRY(ldpc::launch_frames(G, d->st, phys_tile(d), seed, snr_point, sigma, frame0, ldpc::kFramesCh, nullptr,
                                s));
    // export writes u only for j<k, at [f][k]: give it the [count][k] buffer
    HIP_TRY(ldpc::launch_export_frames(G, d->st, u_dev, l_dev, s));
    if (!dev_ptrs) {
        if (u_out) HIP_TRY(hipMemcpyAsync(u_out, u_dev, (size_t)count * G.k, hipMemcpyDeviceToHost, s));
        if (llr_out)
            HIP_TRY(hipMemcpyAsync(llr_out, l_dev, sizeof(double) * (size_t)count * G.n, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(u_dev);
    }
    return LDPC_OK;
}

namespace {

// Streaming tail: the column-parallel VN (launch_vn_tail) replaces vn_kernel
// once at most kTailTiles tiles run; the sub-tile streaming kernel hands its
// frames over once the supply is out and at most LDPC_HANDOFF frames still
// run (default: handoff_frames).  LDPC_TAIL_VN=0 / LDPC_HANDOFF=0 switch them off.
constexpr int kTailTiles = 128;
bool tail_vn_enabled() {
    const char *e = getenv("LDPC_TAIL_VN");
    return !e || atoi(e) != 0;
}
// Default: once the supply is out and at most 3/5 of the slots the sub-tile
// kernel keeps resident (one 16-frame workgroup per CU) still run.  At 3 dB
// (wimax_2304_0.5) that is within a few passes -- about 2/3 of the slots then
// hold frames that will fail, at every stage of their 50 passes -- and the
// step takes 615 ms instead of 1.1 s; at 2 dB, where nearly every slot runs to
// 50 passes, the sub-tile kernel keeps the bulk (3/4: -2 % there;
// profiles/r2au_tail).
// fpw: frames per workgroup of the streaming sub-tile kernel (16, or 8 for
// tile8_stream_kernel), one workgroup per CU.  Round 4, with the
// longest-job-first supply order: the 16-frame kernel hands off as soon as the
// supply is out (every resident frame: 3 dB step 66.3k -> 69.1k cw/s; 3/5 of
// them, 4,000 and "always" measured 66.3k / 68.9k / 68.6k); the 8-frame kernel,
// whose pass is half as long, keeps 3/5 (r3/4A 3 dB: 52.3k vs 47.8k for all
// resident) -- profiles/r4c_ab.
int64_t handoff_frames(int64_t slots, int fpw) {
    const char *e = getenv("LDPC_HANDOFF");
    if (e) return atoll(e);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t resident = std::min<int64_t>(slots, (int64_t)cus * fpw);
    return fpw == 16 ? resident : resident * 3 / 5;
}

// Longest job first (frame_order.hip): the point's frames enter the slots in
// descending syndrome weight of their channel hard decisions, so the frames
// that will run to max_iter start while the slots are still being refilled
// instead of forming a tail after the supply is out.  Counters are sums over
// the point's frames, identical in any order.  LDPC_LPT=0: frame index order.
bool lpt_enabled() {
    const char *e = getenv("LDPC_LPT");
    return !e || atoi(e) != 0;
}
int ensure_order(ldpc_decoder *d, int64_t total) {
    if (d->ord_cap < total) {
        (void)hipFree(d->ord_keys);
        (void)hipFree(d->ord_vals);
        (void)hipFree(d->ord);
        d->ord_keys = nullptr;
        d->ord_vals = d->ord = nullptr;
        d->ord_cap = 0;
        if (int rc = dev_alloc(&d->ord_keys, 2 * (size_t)total)) return rc;
        if (int rc = dev_alloc(&d->ord_vals, (size_t)total)) return rc;
        if (int rc = dev_alloc(&d->ord, (size_t)total)) return rc;
        d->ord_cap = total;
    }
    const size_t tb = ldpc::frame_order_temp_bytes((int)total);
    if (d->ord_tmp_bytes < tb) {
        (void)hipFree(d->ord_tmp);
        d->ord_tmp = nullptr;
        d->ord_tmp_bytes = 0;
        if (hipMalloc(&d->ord_tmp, tb) != hipSuccess)
            return ldpc_fail(LDPC_ENOMEM, "hipMalloc(%zu bytes) failed (frame order scratch)", tb);
        d->ord_tmp_bytes = tb;
    }
    return LDPC_OK;
}

// Streaming schedule of one SNR point: the decoder's cap frames are slots.  A
// slot whose frame finishes (vn_kernel) is refilled with the next frame index
// (refill_kernel), so no slot waits for the slowest frame of its tile or
// chunk; only the last frames of the point form a tail.  Frames, and the
// counters summed over them, are exactly the static schedule's.
int mc_stream_point(ldpc_decoder *d, const DevGraph &G, uint64_t seed, int p, double sigma, int64_t total,
                    int64_t frame0, int max_iter, bool nllr, bool split, hipStream_t s) {
    if (total == 0) return LDPC_OK;
    const int ntiles = (int)std::min<int64_t>(d->cap_tiles, (total + kTile - 1) / kTile);
    const int *order = nullptr;  // supply order (null: frame index order)
    // only when frames wait for a slot: with every frame running from the
    // start the order cannot change when any of them runs.  The split path
    // runs every slot each launch; a tile streaming kernel keeps one
    // workgroup per CU resident (its other workgroups start as those finish)
    int64_t running = (int64_t)ntiles * kTile;
    if (!split && ldpc::use_tile_stream(G)) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const int fpw = G.ef == 8 ? 8 : ldpc::sub_frames(G) == 16 ? 16 : kTile;
        running = std::min<int64_t>(running, (int64_t)cus * fpw);
    }
    if (lpt_enabled() && total > running && total <= INT32_MAX && G.std_form && G.a_packed && G.m <= 65535) {
        if (int rc = ensure_order(d, total)) return rc;
        HIP_TRY(timed(d, LDPC_K_GEN, s, [&] {
            return ldpc::launch_frame_order(G, seed, p, sigma, frame0, (int)total, d->ord_keys, d->ord_vals, d->ord,
                                            d->ord_tmp, d->ord_tmp_bytes, s);
        }));
        order = d->ord;
    }
    state_bind(d, ntiles, ntiles * kTile);
    d->st.order = order;
    DevState st = d->st;
    unsigned long long *ctr = d->counters + (size_t)p * LDPC_MC_NCOUNT;
    unsigned long long *next = d->counters + d->counters_cap;
    const int cap = d->cap_tiles * kTile;
    // streaming tail VN (column-parallel, launch_vn_tail) once few tiles run
    const bool tail_ok = G.a_packed && ((G.k + 31) >> 5) <= 64 && tail_vn_enabled();
    if (tail_ok)
        if (int rc = ensure_tail_bufs(d, s)) return rc;
    auto refill = [&] {
        return timed(d, LDPC_K_GEN, s,
                     [&] { return ldpc::launch_refill(G, st, seed, p, sigma, frame0, total, next, s); });
    };
    int cur = ntiles;  // tiles the steps launch (shrinks as the tail is compacted)
    if (!split && ldpc::use_tile_stream(G) && st.ntiles * tile_scratch_rows(G) <= st.nslots) {
        // one launch: every workgroup's lanes pull frames until the supply is
        // out; the sub-tile decoder hands its last running frames to the
        // column-parallel tail below (one pass of a sub-tile costs ~14 ms)
        const int fpw = G.ef == 8 ? 8 : ldpc::sub_frames(G) == 16 ? 16 : 0;  // 0: tile_stream_kernel, no hand-off
        const int64_t ho = tail_ok && fpw ? handoff_frames((int64_t)ntiles * kTile, fpw) : 0;
        HIP_TRY(hipMemsetAsync(next, 0, sizeof(unsigned long long), s));
        HIP_TRY(timed(d, LDPC_K_TILE, s, [&] {
            return ldpc::launch_tile_stream(G, st, max_iter, nllr, seed, p, sigma, frame0, total, next, ctr, ho, s);
        }));
        if (ho <= 0) return LDPC_OK;
        unsigned long long finished = 0;
        HIP_TRY(hipMemcpyAsync(&finished, ctr, sizeof(finished), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if ((int64_t)finished >= total) return LDPC_OK;
        // the running frames (split-path slot state, written by the kernel)
        // move into the first tiles; the loop below continues them
        const int nt = (int)((total - (int64_t)finished + kTile - 1) / kTile);
        if (!d->cpairs && dev_alloc(&d->cpairs, 1 + 2 * (size_t)cap)) return LDPC_ENOMEM;
        if (nt < cur) {
            HIP_TRY(ldpc::launch_compact(G, st, nt, cap, d->cpairs, s));
            state_bind(d, nt, nt * kTile);
            d->st.order = order;
            st = d->st;
            cur = nt;
        } else {
            HIP_TRY(ldpc::launch_compact(G, st, cur, cap, d->cpairs, s));  // tile_active of every tile
        }
    } else {
        HIP_TRY(ldpc::launch_stream_init(G, st, s));
        HIP_TRY(hipMemsetAsync(next, 0, sizeof(unsigned long long), s));
        HIP_TRY(refill());
    }
    HIP_TRY(hipMemsetAsync(st.rare_count, 0, sizeof(int) * 2, s));  // see run_iterations
    const int64_t slots = (int64_t)ntiles * kTile;
    const int64_t min_steps = (total + slots - 1) / slots;            // every slot needs >= 1 step per frame
    const int64_t max_steps = (min_steps + 1) * (int64_t)max_iter;   // every frame stops by max_iter
    constexpr int kPoll = 4;
    int64_t step = 0;
    const bool compact = [] {
        const char *e = getenv("LDPC_COMPACT");
        return !e || atoi(e) != 0;
    }();
    // compact once live <= cur * 64 * kc / 8 (LDPC_COMPACT_AT, eighths)
    const int kc = [] {
        const char *e = getenv("LDPC_COMPACT_AT");
        return e ? std::max(1, std::min(8, atoi(e))) : 4;
    }();
    const bool tlog = getenv("LDPC_TAIL_LOG") != nullptr;
    for (;;) {
        // every frame fits in the slots: all start now and stop by max_iter
        const int64_t until = total <= slots ? std::max<int64_t>(step + kPoll, max_iter)
                                             : std::max<int64_t>(step + kPoll, min_steps);
        for (; step < until; ++step) {
            const int par = (int)(step & 1);
            HIP_TRY(timed(d, LDPC_K_CN, s, [&] { return ldpc::launch_cn(G, st, par, s, true); }));
            HIP_TRY(ldpc::launch_cn_rare(G, st, par, s, true));
            if (tail_ok && cur <= kTailTiles)
                HIP_TRY(timed(d, LDPC_K_VN_COLS, s,
                              [&] { return ldpc::launch_vn_tail(G, st, max_iter, nllr, d->tzb, d->tcnt, ctr, s); }));
            else
                HIP_TRY(timed(d, LDPC_K_VN, s, [&] { return ldpc::launch_vn(G, st, 0, max_iter, nllr, s, ctr); }));
            HIP_TRY(refill());
        }
        unsigned long long finished = 0, handed = 0;
        HIP_TRY(hipMemcpyAsync(&finished, ctr, sizeof(finished), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&handed, next, sizeof(handed), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if ((int64_t)finished >= total) return LDPC_OK;
        // tail: the supply is out and at most half of the launched slots
        // still run -> move them into the first tiles and launch only those
        const int64_t live = std::min<int64_t>((int64_t)handed, total) - (int64_t)finished;
        if (tlog) fprintf(stderr, "[tail] step %lld cur %d live %lld\n", (long long)step, cur, (long long)live);
        const int nt = (int)((live + kTile - 1) / kTile);
        if (compact && (int64_t)handed >= total && cur > 1 && live > 0 && nt < cur &&
            live * 8 <= (int64_t)cur * kTile * kc) {
            if (!d->cpairs && dev_alloc(&d->cpairs, 1 + 2 * (size_t)cap)) return LDPC_ENOMEM;
            HIP_TRY(ldpc::launch_compact(G, st, nt, cap, d->cpairs, s));
            state_bind(d, nt, nt * kTile);
            d->st.order = order;
            st = d->st;
            cur = nt;
        }
        if (step > max_steps)
            return ldpc_fail(LDPC_EDEVICE, "ldpc_mc_run: streaming schedule did not drain (%llu of %lld frames)",
                             finished, (long long)total);
    }
}

}  // namespace

int ldpc_frame_order(ldpc_decoder *d, uint64_t seed, int32_t snr_point, double sigma, int64_t frame0,
                     int32_t count, int32_t *order_out, void *stream) {
    if (!d || count < 0 || snr_point < 0 || frame0 < 0 || !(sigma > 0.0) || (count > 0 && !order_out))
        return ldpc_fail(LDPC_EINVAL, "ldpc_frame_order: bad arguments");
    const DevGraph &G = d->g->dg;
    if (!G.std_form || !G.a_packed || G.m > 65535)
        return ldpc_fail(LDPC_EINVAL, "ldpc_frame_order: graph is not [A | I_m] with m <= 65535");
    if (count == 0) return LDPC_OK;
    DeviceGuard dg(d->g->device);
    hipStream_t s = (hipStream_t)stream;
    if (int rc = ensure_order(d, count)) return rc;
    HIP_TRY(ldpc::launch_frame_order(G, seed, snr_point, sigma, frame0, count, d->ord_keys, d->ord_vals, d->ord,
                                     d->ord_tmp, d->ord_tmp_bytes, s));
    HIP_TRY(hipMemcpyAsync(order_out, d->ord, sizeof(int32_t) * (size_t)count, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return LDPC_OK;
}

int ldpc_mc_run(ldpc_decoder *d, uint64_t seed, int32_t n_points, const double *sigmas, int64_t frames_per_point,
                int64_t frame0, int32_t max_iter, uint32_t flags, int64_t *counters_out, void *stream) {
    if (!d || n_points <= 0 || !sigmas || frames_per_point < 0 || frame0 < 0 || max_iter < 1 || !counters_out)
        return ldpc_fail(LDPC_EINVAL, "ldpc_mc_run: bad arguments");
    const DevGraph G = call_graph(d, flags);
    if (!G.std_form) return ldpc_fail(LDPC_EINVAL, "ldpc_mc_run: graph is not [A | I_m]");
    for (int p = 0; p < n_points; ++p)
        if (!(sigmas[p] > 0.0)) return ldpc_fail(LDPC_EINVAL, "ldpc_mc_run: sigma[%d] <= 0", p);
    DeviceGuard dg(d->g->device);
    if (int rc0 = ensure_messages(d)) return rc0;
    hipStream_t s = (hipStream_t)stream;
    const bool nllr = flags & LDPC_F_NLLR;
    const int need = n_points * LDPC_MC_NCOUNT;
    if (d->counters_cap < need) {
        (void)hipFree(d->counters);
        d->counters = nullptr;
        d->counters_cap = 0;
        if (int rc = dev_alloc(&d->counters, (size_t)need + 1)) return rc;
        d->counters_cap = need;
    }
    HIP_TRY(hipMemsetAsync(d->counters, 0, sizeof(unsigned long long) * need, s));
    const int64_t cap = (int64_t)d->cap_tiles * kTile;
    if (!(flags & LDPC_F_STATIC)) {
        for (int p = 0; p < n_points; ++p)
            if (int rc = mc_stream_point(d, G, seed, p, sigmas[p], frames_per_point, frame0, max_iter, nllr,
                                         flags & LDPC_F_SPLIT, s))
                return rc;
    } else {
        if (int rc = ensure_pbits(d, G)) return rc;
        for (int p = 0; p < n_points; ++p) {
            for (int64_t start = 0; start < frames_per_point; start += cap) {
                const int cnt = (int)std::min<int64_t>(cap, frames_per_point - start);
                state_bind(d, (cnt + kTile - 1) / kTile, cnt);
                HIP_TRY(ldpc::launch_reset(G, d->st, s));
                const DevState st = d->st;
                HIP_TRY(timed(d, LDPC_K_GEN, s,
                              [&] { return ldpc::launch_frames(G, st, phys_tile(d), seed, p, sigmas[p], frame0 + start,
                                                               ldpc::kFramesCh, nullptr, s); }));
                if (int rc = run_iterations(d, G, st, max_iter, nllr, s, true, flags & LDPC_F_SPLIT)) return rc;
                HIP_TRY(timed(d, LDPC_K_COUNT, s, [&] {
                    return ldpc::launch_count(G, st, d->counters + (size_t)p * LDPC_MC_NCOUNT, s);
                }));
            }
        }
    }
    std::vector<unsigned long long> h(need);
    HIP_TRY(hipMemcpyAsync(h.data(), d->counters, sizeof(unsigned long long) * need, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int i = 0; i < need; ++i) counters_out[i] = (int64_t)h[i];
    return LDPC_OK;
}

int ldpc_rare_rows_read(ldpc_decoder *d, int64_t *out) {
    if (!d || !out) return ldpc_fail(LDPC_EINVAL, "ldpc_rare_rows_read: bad arguments");
    DeviceGuard dg(d->g->device);
    int h[2] = {0, 0};
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(h, d->rare + 2, sizeof h, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(d->rare + 2, 0, sizeof h));
    out[0] = h[0];
    out[1] = h[1];
    return LDPC_OK;
}

// ---------------------------------------------------------- physical mode
namespace {

constexpr size_t kLdsLimit = 160 * 1024 - 1024;

int phys_grid(const DevGraph &G) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
    }
    const size_t lds = ldpc::phys_lds_bytes(G) + 64;
    const int waves = ldpc::phys_block_threads(G) / 64;  // <= 32 waves / CU
    int per_cu = (int)std::min<size_t>(32 / waves, kLdsLimit / lds);
    if (per_cu < 1) per_cu = 1;
    return cus * per_cu;
}


}  // namespace

int64_t ldpc_phys_lds_bytes(const ldpc_graph *g) { return g ? (int64_t)ldpc::phys_lds_bytes(g->dg) : -1; }

namespace {

int phys_decode_lds(const ldpc_graph *g, int32_t batch, const double *llr, int32_t max_iter, uint32_t flags,
                    uint8_t *z_out, int32_t *conv_out, int32_t *status_out, int32_t *iters_out, float *post_out,
                    hipStream_t s) {
    const DevGraph &G = g->dg;
    const size_t n = (size_t)G.n, B = (size_t)batch;
    if (flags & LDPC_F_DEVICE_PTRS) {
        HIP_TRY(ldpc::launch_phys(G, llr, nullptr, 0, batch, max_iter, z_out, conv_out, status_out, iters_out, post_out,
                                  nullptr, nullptr, std::min(phys_grid(G), batch), s));
        return LDPC_OK;
    }
    double *d_llr = nullptr;
    uint8_t *d_z = nullptr;
    int *d_i = nullptr;
    float *d_post = nullptr;
    int rc = dev_alloc(&d_llr, B * n);
    if (!rc) rc = dev_alloc(&d_z, B * n);
    if (!rc) rc = dev_alloc(&d_i, 3 * B);
    if (!rc && post_out) rc = dev_alloc(&d_post, B * n);
    hipError_t e = hipSuccess;
    if (!rc) {
        e = hipMemcpyAsync(d_llr, llr, sizeof(double) * B * n, hipMemcpyHostToDevice, s);
        if (!e) e = ldpc::launch_phys(G, d_llr, nullptr, 0, batch, max_iter, d_z, d_i, d_i + B, d_i + 2 * B, d_post, nullptr,
                                     nullptr, std::min(phys_grid(G), batch), s);
        if (!e && z_out) e = hipMemcpyAsync(z_out, d_z, B * n, hipMemcpyDeviceToHost, s);
        if (!e && conv_out) e = hipMemcpyAsync(conv_out, d_i, sizeof(int) * B, hipMemcpyDeviceToHost, s);
        if (!e && status_out) e = hipMemcpyAsync(status_out, d_i + B, sizeof(int) * B, hipMemcpyDeviceToHost, s);
        if (!e && iters_out) e = hipMemcpyAsync(iters_out, d_i + 2 * B, sizeof(int) * B, hipMemcpyDeviceToHost, s);
        if (!e && post_out) e = hipMemcpyAsync(post_out, d_post, sizeof(float) * B * n, hipMemcpyDeviceToHost, s);
        if (!e) e = hipStreamSynchronize(s);
        if (e) rc = ldpc_fail(LDPC_EDEVICE, "ldpc_phys_decode: %s", hipGetErrorString(e));
    }
    (void)hipFree(d_llr);
    (void)hipFree(d_z);
    (void)hipFree(d_i);
    (void)hipFree(d_post);
    return rc;
}

// Decode the frames bound in d->st (channel LLRs in d->ch) on graph P with the
// HBM-resident tile kernels: up to max_iter CN+VN sweeps, then a syndrome-only
// sweep.  The host reads the running-tile and running-frame counts after
// VN(it) for it < 4 and every 4th iteration after, and stops issuing sweeps
// once they are zero.  With ctr (a Monte-Carlo run: only the counters leave
// the device) the running frames are compacted into the first tiles once at
// most a quarter of the launched slots hold them, the finished frames counted
// into ctr first (phys_tile.hip).
int phys_tile_decode(ldpc_decoder *d, const DevGraph &P, int max_iter, bool from_ch, hipStream_t s,
                     unsigned long long *ctr = nullptr) {
    if (d->pactive_cap < 2 * max_iter) {
        (void)hipFree(d->pactive);
        d->pactive = nullptr;
        d->pactive_cap = 0;
        if (int rc = dev_alloc(&d->pactive, 2 * (size_t)max_iter)) return rc;
        d->pactive_cap = 2 * max_iter;
    }
    DevState st = d->st;  // st.ntiles shrinks with each compaction
    const PhysTile pt = phys_tile(d);
    const int cap = d->cap_tiles * kTile;
    // LDPC_PHYS_COMPACT=0: no compaction (A/B, diagnosis; the counters are the same)
    const bool compact = [] {
        const char *e = getenv("LDPC_PHYS_COMPACT");
        return !e || atoi(e) != 0;
    }();
    HIP_TRY(hipMemsetAsync(d->pactive, 0, sizeof(int) * 2 * max_iter, s));
    HIP_TRY(ldpc::launch_phys_tile_init(P, st, pt, from_ch, s));
    for (int it = 0; it < max_iter; ++it) {
        HIP_TRY(timed(d, LDPC_K_PHYS_CN, s, [&] { return ldpc::launch_phys_tile_cn(P, st, pt, it, false, s); }));
        HIP_TRY(timed(d, LDPC_K_PHYS_VN, s,
                      [&] { return ldpc::launch_phys_tile_vn(P, st, pt, it, d->pactive, max_iter, s); }));
        if (it + 1 < max_iter && (it < 4 || (it + 1) % 4 == 0)) {
            // iterations 1 and 2: the frames whose posterior already
            // satisfies every check stop now instead of after the next CN
            // sweep (DVB-S2 profile at 1 dB, 2 iterations per frame: +25 %).
            // Each early syndrome costs ~1 ms on 128 tiles, more than it saves
            // where frames stop after 20-40 iterations (the -2.5 dB
            // waterfall: -1.4 % with it at every poll of it < 4,
            // profiles/r5_ab/r5ao_ab)
            if (it == 1 || it == 2)
                HIP_TRY(timed(d, LDPC_K_PHYS_VN, s, [&] {
                    return ldpc::launch_phys_tile_early_exit(P, st, pt, it, d->pactive, max_iter, s);
                }));
            int running[2] = {0, 0};  // tiles, frames
            HIP_TRY(hipMemcpyAsync(&running[0], d->pactive + it, sizeof(int), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(&running[1], d->pactive + max_iter + it, sizeof(int), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (running[0] == 0) break;  // every frame has stopped (converged; final() leaves them alone)
            const int nt = (running[1] + kTile - 1) / kTile;
            // (a quarter: half measured the same, profiles/r5_ab/r5am_ab)
            if (ctr && compact && nt < st.ntiles && 4 * (int64_t)running[1] <= (int64_t)st.ntiles * kTile) {
                if (!d->cpairs && dev_alloc(&d->cpairs, 1 + 2 * (size_t)cap)) return LDPC_ENOMEM;
                HIP_TRY(timed(d, LDPC_K_COUNT, s, [&] { return ldpc::launch_phys_tile_count(P, st, pt, ctr, s); }));
                HIP_TRY(ldpc::launch_phys_compact(P, st, pt, nt, cap, d->cpairs, s));
                st.ntiles = nt;
            }
        }
    }
    HIP_TRY(ldpc::launch_phys_tile_cn(P, st, pt, max_iter, true, s));
    HIP_TRY(ldpc::launch_phys_tile_final(P, st, pt, max_iter, s));
    return LDPC_OK;
}

bool phys_use_lds(const DevGraph &P, uint32_t flags) {
    return !(flags & LDPC_F_PHYS_HBM) && ldpc::phys_lds_bytes(P) <= kLdsLimit;
}

int phys_decode_tile(const ldpc_graph *g, int32_t batch, const double *llr, int32_t max_iter, uint32_t flags,
                     uint8_t *z_out, int32_t *conv_out, int32_t *status_out, int32_t *iters_out, float *post_out,
                     hipStream_t s) {
    const DevGraph &G = g->dg;
    const bool dev_ptrs = flags & LDPC_F_DEVICE_PTRS;
    const int chunk = std::min<int>(batch, 1024);
    ldpc_decoder *d = nullptr;
    if (int rc = ldpc_decoder_create(g, chunk, &d)) return rc;
    struct Free {
        ldpc_decoder *d;
        ~Free() { ldpc_decoder_destroy(d); }
    } guard{d};
    if (int rc = ensure_phys_tile(d, G)) return rc;
    const size_t n = (size_t)G.n;
    for (int start = 0; start < batch; start += chunk) {
        const int cnt = std::min(chunk, batch - start);
        state_bind(d, (cnt + kTile - 1) / kTile, cnt);
        const DevState &st = d->st;
        const double *src = llr + (size_t)start * n;
        if (!dev_ptrs) {
            HIP_TRY(hipMemcpyAsync(d->llr_stage, src, sizeof(double) * cnt * n, hipMemcpyHostToDevice, s));
            src = d->llr_stage;
        }
        HIP_TRY(ldpc::launch_load_llr(G, st, src, s));
        if (int rc = phys_tile_decode(d, G, max_iter, true, s)) return rc;
        uint8_t *zd = z_out ? (dev_ptrs ? z_out + (size_t)start * n : d->z_stage) : nullptr;
        float *pd = post_out ? (dev_ptrs ? post_out + (size_t)start * n : (float *)d->post_stage) : nullptr;
        HIP_TRY(ldpc::launch_phys_tile_out(G, st, phys_tile(d), zd, pd, s));
        const hipMemcpyKind kind = dev_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        if (conv_out) HIP_TRY(hipMemcpyAsync(conv_out + start, st.conv, sizeof(int) * cnt, kind, s));
        if (status_out) HIP_TRY(hipMemcpyAsync(status_out + start, st.status, sizeof(int) * cnt, kind, s));
        if (iters_out) HIP_TRY(hipMemcpyAsync(iters_out + start, st.iters, sizeof(int) * cnt, kind, s));
        if (!dev_ptrs) {
            if (z_out) HIP_TRY(hipMemcpyAsync(z_out + (size_t)start * n, zd, cnt * n, hipMemcpyDeviceToHost, s));
            if (post_out)
                HIP_TRY(hipMemcpyAsync(post_out + (size_t)start * n, pd, sizeof(float) * cnt * n,
                                       hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(hipStreamSynchronize(s));  // staging and workspace are reused / freed
    }
    return LDPC_OK;
}

}  // namespace

int ldpc_phys_decode(const ldpc_graph *g, int32_t batch, const double *llr, int32_t max_iter, uint32_t flags,
                     uint8_t *z_out, int32_t *conv_out, int32_t *status_out, int32_t *iters_out, float *post_out,
                     void *stream) {
    if (!g) return ldpc_fail(LDPC_EINVAL, "ldpc_phys_decode: NULL graph");
    if (batch < 0 || max_iter < 1 || (batch > 0 && !llr))
        return ldpc_fail(LDPC_EINVAL, "ldpc_phys_decode: bad arguments (batch=%d max_iter=%d)", batch, max_iter);
    if (batch == 0) return LDPC_OK;
    DeviceGuard dg(g->device);
    hipStream_t s = (hipStream_t)stream;
    if (phys_use_lds(g->dg, flags))
        return phys_decode_lds(g, batch, llr, max_iter, flags, z_out, conv_out, status_out, iters_out, post_out, s);
    return phys_decode_tile(g, batch, llr, max_iter, flags, z_out, conv_out, status_out, iters_out, post_out, s);
}

int ldpc_phys_mc_run(ldpc_decoder *d, const ldpc_graph *gp, uint64_t seed, int32_t n_points, const double *sigmas,
                     int64_t frames_per_point, int64_t frame0, int32_t max_iter, uint32_t flags, int64_t *counters_out,
                     void *stream) {
    if (!gp) return ldpc_fail(LDPC_EINVAL, "ldpc_phys_mc_run: NULL graph");
    if (!d || n_points <= 0 || !sigmas || frames_per_point < 0 || frame0 < 0 || max_iter < 1 || !counters_out)
        return ldpc_fail(LDPC_EINVAL, "ldpc_phys_mc_run: bad arguments");
    const DevGraph &G = d->g->dg;
    const DevGraph &P = gp->dg;
    if (!G.std_form && !(G.ira && d->g == gp))
        return ldpc_fail(LDPC_EINVAL,
                         "ldpc_phys_mc_run: the decoder's graph must be the code's H_std = [A | I_m], or the "
                         "IRA graph itself");
    if (P.n != G.n || P.k != G.k)
        return ldpc_fail(LDPC_EINVAL, "ldpc_phys_mc_run: physical graph shape %dx%d != %dx%d", P.m, P.n, G.m, G.n);
    for (int p = 0; p < n_points; ++p)
        if (!(sigmas[p] > 0.0)) return ldpc_fail(LDPC_EINVAL, "ldpc_phys_mc_run: sigma[%d] <= 0", p);
    DeviceGuard dg(d->g->device);
    hipStream_t s = (hipStream_t)stream;
    const bool lds = phys_use_lds(P, flags);
    if (!lds)
        if (int rc = ensure_phys_tile(d, P)) return rc;
    if (int rc = ensure_pbits(d, G)) return rc;
    const int need = n_points * LDPC_MC_NCOUNT;
    if (d->counters_cap < need) {
        (void)hipFree(d->counters);
        d->counters = nullptr;
        d->counters_cap = 0;
        if (int rc = dev_alloc(&d->counters, (size_t)need + 1)) return rc;
        d->counters_cap = need;
    }
    HIP_TRY(hipMemsetAsync(d->counters, 0, sizeof(unsigned long long) * need, s));
    const int64_t cap = (int64_t)d->cap_tiles * kTile;
    for (int p = 0; p < n_points; ++p) {
        unsigned long long *ctr = d->counters + (size_t)p * LDPC_MC_NCOUNT;
        for (int64_t start = 0; start < frames_per_point; start += cap) {
            const int cnt = (int)std::min<int64_t>(cap, frames_per_point - start);
            state_bind(d, (cnt + kTile - 1) / kTile, cnt);
            const DevState st = d->st;
            // frames go straight to the decoder's fp32 Lambda: tile layout for the
            // HBM tile decoder, row-major (contiguous per frame) for the LDS decoder
            float *rows = (float *)d->llr_stage;  // cap x n doubles: room for cap x n floats
            HIP_TRY(timed(d, LDPC_K_GEN, s, [&] {
                return ldpc::launch_frames(G, st, phys_tile(d), seed, p, sigmas[p], frame0 + start,
                                           lds ? ldpc::kFramesRowLambda : ldpc::kFramesTileLambda, rows, s);
            }));
            if (lds) {
                HIP_TRY(timed(d, LDPC_K_PHYS, s, [&] {
                    return ldpc::launch_phys(P, nullptr, rows, 2, cnt, max_iter, nullptr, nullptr, nullptr, nullptr,
                                             nullptr, st.ubits, ctr, std::min(phys_grid(P), cnt), s);
                }));
            } else {
                if (int rc = phys_tile_decode(d, P, max_iter, false, s, ctr)) return rc;
                HIP_TRY(timed(d, LDPC_K_COUNT, s,
                              [&] { return ldpc::launch_phys_tile_count(P, st, phys_tile(d), ctr, s); }));
            }
        }
    }
    std::vector<unsigned long long> h(need);
    HIP_TRY(hipMemcpyAsync(h.data(), d->counters, sizeof(unsigned long long) * need, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int i = 0; i < need; ++i) counters_out[i] = (int64_t)h[i];
    return LDPC_OK;
}

// -------------------------------------------------------------- profiling
int ldpc_profile_enable(ldpc_decoder *d, int enable) {
    if (!d) return ldpc_fail(LDPC_EINVAL, "ldpc_profile_enable: NULL decoder");
    d->prof = enable != 0;
    return LDPC_OK;
}

int ldpc_profile_read(ldpc_decoder *d, double *ms_out, int64_t *launches_out) {
    if (!d) return ldpc_fail(LDPC_EINVAL, "ldpc_profile_read: NULL decoder");
    DeviceGuard dg(d->g->device);
    double ms[LDPC_K_NKINDS] = {};
    int64_t cnt[LDPC_K_NKINDS] = {};
    for (auto &sp : d->spans) {
        HIP_TRY(hipEventSynchronize(sp.b));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, sp.a, sp.b));
        ms[sp.kind] += t;
        cnt[sp.kind] += 1;
        d->pool.push_back(sp.a);
        d->pool.push_back(sp.b);
    }
    d->spans.clear();
    for (int i = 0; i < LDPC_K_NKINDS; ++i) {
        if (ms_out) ms_out[i] = ms[i];
        if (launches_out) launches_out[i] = cnt[i];
    }
    return LDPC_OK;
}

}  // extern "C"
