// spa_device.h -- device-side layout and kernel entry points of libldpc_hip.so.
//
// Data layout in HBM ("frame tiles"): 64 frames form one tile, one frame per
// lane of a wavefront.  Every per-edge / per-column array is stored
// [tile][item][64 lanes], so a wavefront touching item i of its tile reads
// 64 consecutive doubles (512 contiguous bytes): fully coalesced, with no
// index math per lane.
//   E   [tile][nnz][64]  fp64 check->variable messages (CSR edge order of H_std);
//                        for tile8.hip's graphs [tile][8][nnz][8] (e_base below)
//   T   [slot][max_row_deg][64] fp64 scratch of cn_rare_kernel (slot = its
//                        global wavefront id; nslots = 4 x its grid)
//   L   [tile][n][64]    fp64 a-posteriori LLRs
//   ch  [tile][n][64]    fp64 channel LLRs
//   ub  [tile][kw][64]   info bits (Monte-Carlo path), kw = ceil(k/32)
// Per frame: done / conv / status / iters / nllr count (+ fresh / refill of the
// streaming Monte-Carlo schedule); per tile: active flag.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldpc {

constexpr int kTile = 64;  // frames per tile == wavefront width on CDNA

// wavefronts per sub-tile workgroup (tile_sub.hip); the host builds the
// P3 order table (DevGraph::p3dep) for this chunking
constexpr int kSubWaves = 16;
// message-array slack (edges x 64 lanes) past the last tile: the sub-tile
// decoder's unclamped slot loads overshoot a row by < Q*K = 64 edges
constexpr int kEPadEdges = 128;

struct DevGraph {
    int m, n, k, nnz;
    int max_row_deg, max_col_deg;
    int std_form;            // 1 if H_std = [A | I_m] exactly (encoder usable)
    int ira;                 // 1 if H = [H_info | staircase] (IRA encoder usable)
    const int *row_ptr;      // [m+1]
    const int *col_idx;      // [nnz]
    const int *csc_ptr;      // [n+1]
    const int *csc_edge;     // [nnz] CSR edge id, rows ascending within a column
    const int *csc_row;      // [nnz] row of that edge
    const uint32_t *a_packed;  // [m][kw] bit j of row r = A[r][j] (encoder; std_form only)
    const int *p3dep;          // [m][16] sub-tile S order: lo | hi << 8 (tile_sub.hip sub_p3)
    const int *p3dep8;         // [m][16] the same over each row's A edges (tile8.hip: identity excluded)
    int ef;                    // frames per E block (64, or 8 for tile8.hip's graphs): e_base
    int t8pair;                // tile8.hip runs its pair form (two rows per wavefront) on this graph
    int lpt_weak_id;           // frame_order.hip: rank equal syndromes by the weakest identity bit of an
                               // odd-degree row (set when at most half the rows have odd degree)
    int zinj;                  // test-only erasure injection of the frame source (LDPC_F_TEST_ZERO): 0 = off,
                               // else frame_source.h test_zero_llr (set per call, never on the graph itself)
};

// E layout inside a tile: the 64 frames in blocks of g.ef, each block
// [nnz][ef], so a workgroup that decodes ef frames reads whole cache lines
// (ef = 64: [tile][nnz][64]; ef = 8: [tile][8][nnz][8], the 8-frame sub-tile
// decoder of tile8.hip).  Element (tile, e, lane) = E[e_base(tile, lane) + e * ef].
__host__ __device__ inline size_t e_base(const DevGraph &g, int tile, int lane) {
    return (size_t)tile * g.nnz * kTile + (size_t)(lane / g.ef) * g.nnz * g.ef + (size_t)(lane % g.ef);
}

struct DevState {
    double *E, *T, *L, *ch;
    int *done, *conv, *status, *iters, *nllr_cnt;
    int *tile_active;
    int *fresh, *refill;     // streaming Monte-Carlo: lane holds a new frame / lane wants one
    const int *order;        // streaming Monte-Carlo: local frame index of supply position i (frame_order.hip:
                             // heaviest syndrome first), or null: frame index order
    int *rare_list;          // [ntiles*m] tile*m+row of rows left to cn_rare_kernel
    int *rare_count;         // [2] per iteration parity, then two running totals (ldpc_rare_rows_read):
                             // [2] rows cn_rare_kernel took, [3] rare rows the tile decoders took in-kernel
    int *active_count;       // [max_iter] or null: vn_kernel adds the tiles still running after it
    int nslots;
    uint32_t *ubits;         // MC only (may be null)
    double *nllr_hist;       // [frame][hist_stride] or null
    int hist_stride;
    int ntiles;              // tiles in this chunk
    int count;               // valid frames in this chunk
};

// Physical mode with HBM-resident state (phys_tile.hip), same tile layout.
struct PhysTile {
    float *E;          // [tile][nnz][64] check->variable messages
    float *L;          // [tile][n][64] posteriors (Lambda convention: L < 0 -> bit 1)
    float *Lam;        // [tile][n][64] Lambda = -channel LLR
    int *bad;          // [2][cap] row-syndrome flags, by iteration parity
    uint32_t *pbits;   // [tile][m/32][64] IRA: in-word prefix XOR of s = H_info u (generator scratch)
    uint32_t *wpar;    // [tile][m/1024][64] IRA: bit w = parity of s words before w
    int cap;           // frames of capacity (stride of bad)
    uint8_t *zb;       // [tile][ceil(n/8)][64] hard-decision bits of the last VN sweep (bit j&7 of byte j>>3: L < 0)
};

// --- launchers (spa_kernels.hip); all asynchronous on `s` ---
hipError_t launch_reset(const DevGraph &g, const DevState &st, hipStream_t s);
hipError_t launch_load_llr(const DevGraph &g, const DevState &st, const double *llr, hipStream_t s);
// stream = the streaming Monte-Carlo schedule (lanes at different iterations,
// see refill_kernel); stream_ctr != null selects the streaming VN.
hipError_t launch_cn(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream = false);
bool use_cn_row(const DevGraph &g);  // launch_cn runs cn_row_kernel (else cn_kernel)
hipError_t launch_cn_rare(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream = false);
hipError_t launch_vn(const DevGraph &g, const DevState &st, int it, int max_iter, bool nllr, hipStream_t s,
                     unsigned long long *stream_ctr = nullptr);
// tile-resident decoder (tile_kernels.hip): all iterations of a tile in one
// workgroup, check- and variable-node updates fused; [A | I_m] graphs whose A
// column sums fit in LDS (tile_lds_bytes > 0).  Needs st.ntiles <= st.nslots.
// Codes whose column sums of 64 frames do not fit (the WiMAX 2304 codes) run
// the sub-tile decoder (tile_sub.hip: 16 or 8 frames per workgroup).
size_t tile_lds_bytes(const DevGraph &g);
const char *tile_kernel_name(const DevGraph &g);  // "tile_kernel", "tile_sub_kernel" or ""
bool use_tile(const DevGraph &g);
hipError_t launch_tile(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s);
// Streaming Monte-Carlo through the tile-resident decoder (one launch per SNR
// point; LDPC_TILE_STREAM=0 keeps the split CN/VN/refill loop).
bool use_tile_stream(const DevGraph &g);
// handoff > 0 (the 16- and 8-frame sub-tile decoders): the kernel stops once
// the supply is out and at most `handoff` frames still run, leaving them as
// split-path slot state (done / iters / fresh; E, L, ch, ubits in place)
hipError_t launch_tile_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                              int snr_point, double sigma, int64_t frame0, int64_t total, unsigned long long *next,
                              unsigned long long *ctr, int64_t handoff, hipStream_t s);
// 8-frame sub-tile decoder (tile8.hip): the WiMAX 2304 codes; its graphs keep
// E in 8-frame blocks (DevGraph::ef = 8, chosen at graph creation)
bool tile8_applies(const DevGraph &g);
// whether tile8.hip's pair form can run this graph (set DevGraph::t8pair from it at graph creation)
bool tile8_pair_fits(const DevGraph &g);
size_t tile8_lds_bytes(const DevGraph &g);
// rare-row scratch rows per tile it needs: 2, or 4 for its pair form (two alternating
// rare-row buffers per row slot)
int tile8_scratch_per_tile(const DevGraph &g);
hipError_t launch_tile8(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s);
// its streaming Monte-Carlo form (one persistent launch per SNR point, handoff as launch_tile_stream)
size_t tile8_stream_lds_bytes(const DevGraph &g);
hipError_t launch_tile8_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                               int snr_point, double sigma, int64_t frame0, int64_t total, unsigned long long *next,
                               unsigned long long *ctr, int64_t handoff, hipStream_t s);
size_t tile64_lds_bytes(const DevGraph &g);  // tile_kernel (64 frames per workgroup), 0 if it does not apply
int sub_frames(const DevGraph &g);
size_t sub_lds_bytes(const DevGraph &g);
hipError_t launch_tile_sub(const DevGraph &g, const DevState &st, int max_iter, bool nllr, hipStream_t s);
hipError_t launch_tile_sub_stream(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint64_t seed,
                                  int snr_point, double sigma, int64_t frame0, int64_t total,
                                  unsigned long long *next, unsigned long long *ctr, int64_t handoff, hipStream_t s);
hipError_t launch_stream_init(const DevGraph &g, const DevState &st, hipStream_t s);
// streaming tail (few tiles): column-parallel VN + per-tile syndrome/exits,
// the same frames' results and counters as launch_vn(stream).  zb
// [cap_tiles][ceil(n/32)][64] u32 and cnt [cap_tiles*64] int, all zero on entry
// (left zero on exit); std_form graphs with k <= 2048
hipError_t launch_vn_tail(const DevGraph &g, const DevState &st, int max_iter, bool nllr, uint32_t *zb, int *cnt,
                          unsigned long long *ctr, hipStream_t s);
hipError_t launch_vn_cols_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                 int *cnt, hipStream_t s);
// tail_exit_kernel's decode exits; gbad (null: the kernel forms the syndrome
// itself) holds the per-frame row-parity flags of syn_kernel, cleared after use
hipError_t launch_tail_exit_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                   int *cnt, int *gbad, hipStream_t s);
// few-frame decode path (edge_kernels.hip): lanes over a row's / column's
// edges, frame after frame; bit-identical to launch_cn + launch_cn_rare and
// launch_vn_cols_decode.  Rows and columns of up to edge_max_deg() edges;
// gbad [cap_tiles*64] int, zero on entry (left zero)
int edge_max_deg();
hipError_t launch_cn_edge(const DevGraph &g, const DevState &st, int it, hipStream_t s);
hipError_t launch_vn_edge_decode(const DevGraph &g, const DevState &st, int it, bool last, bool nllr, uint32_t *zb,
                                 int *cnt, int *gbad, hipStream_t s);
// split CN on 16-frame sub-tiles, t in registers (cn_sub.hip): rows of the
// 2304 codes; 0 when no shape fits the graph
int cn_sub_shape(const DevGraph &g);
hipError_t launch_cn_sub(const DevGraph &g, const DevState &st, int it, hipStream_t s, bool stream);
// rare-row list entries (cn_rare_kernel): tile * m + row in bits 0..27, and
// in bits 28..31 the 16-frame sub-tiles of the tile it covers (0 = all 64
// frames: cn_kernel / cn_row_kernel; bit s = frames 16 s .. 16 s + 15: cn_sub_kernel)
__host__ __device__ inline uint32_t rare_code(int tile_row, uint32_t subs) {
    return (uint32_t)tile_row | (subs << 28);
}
// supply order of a streamed point (frame_order.hip): keys 2 x total uint32,
// vals total int scratch, order total int out, temp frame_order_temp_bytes
size_t frame_order_temp_bytes(int total);
hipError_t launch_frame_order(const DevGraph &g, uint64_t seed, int snr_point, double sigma, int64_t frame0,
                              int total, uint32_t *keys, int *vals, int *order, void *temp, size_t temp_bytes,
                              hipStream_t s);
// the global frame index of supply position idx of a point starting at frame0
__device__ __forceinline__ long long supply_frame(const DevState &st, int64_t frame0, int64_t idx) {
    return (long long)(frame0 + (st.order ? (int64_t)st.order[idx] : idx));
}
hipError_t launch_refill(const DevGraph &g, const DevState &st, uint64_t seed, int snr_point, double sigma,
                         int64_t frame0, int64_t total, unsigned long long *next, hipStream_t s);
// streaming tail: move the frames running in tiles >= nt into finished slots
// of tiles < nt (pairs: 1 + 2 cap ints of scratch)
hipError_t launch_compact(const DevGraph &g, const DevState &st, int nt, int cap, int *pairs, hipStream_t s);
// the plan alone (phys_tile.hip's compaction moves its own arrays)
hipError_t launch_compact_plan(const DevState &st, int nt, int cap, int *pairs, hipStream_t s);
hipError_t launch_finalize(const DevGraph &g, const DevState &st, uint8_t *z, double *post,
                           hipStream_t s);
hipError_t launch_export_msgs(const DevGraph &g, const DevState &st, double *out, hipStream_t s);
hipError_t launch_export_frames(const DevGraph &g, const DevState &st, uint8_t *u_out, double *llr_out,
                                hipStream_t s);
hipError_t launch_count(const DevGraph &g, const DevState &st, unsigned long long *counters,
                        hipStream_t s);

// physical mode (phys_kernels.hip)
size_t phys_lds_bytes(const DevGraph &g);
int phys_block_threads(const DevGraph &g);  // threads per workgroup launch_phys uses
// layout 0: llr [count][n] fp64; 1: llr = ch tile layout; 2: lam [count][n] fp32 Lambda
hipError_t launch_phys(const DevGraph &g, const double *llr, const float *lam, int layout, int count, int max_iter,
                       uint8_t *z, int *conv, int *status, int *iters, float *post, const uint32_t *ubits,
                       unsigned long long *ctr, int grid, hipStream_t s);

// physical mode, HBM-resident tiles + IRA frame source (phys_tile.hip)
// on-device frames of a chunk (frame_kernels.hip): info bits -> st.ubits,
// parities via pt.pbits/pt.wpar (H_std [A|I] or IRA graph), channel LLRs as
enum FramesOut {
    kFramesCh = 0,          // st.ch, fp64 tile layout (parity decoder, export)
    kFramesTileLambda = 1,  // pt.Lam and pt.L, fp32 tile layout (physical tile decoder)
    kFramesRowLambda = 2,   // row_out [count][n] fp32 Lambda (physical LDS decoder)
};
hipError_t launch_frames(const DevGraph &g, const DevState &st, const PhysTile &pt, uint64_t seed, int snr_point,
                         double sigma, int64_t frame0, FramesOut out, float *row_out, hipStream_t s);
// convert: L = Lambda = -(float)ch (else the generator already wrote them)
hipError_t launch_phys_tile_init(const DevGraph &g, const DevState &st, const PhysTile &pt, bool convert,
                                 hipStream_t s);
hipError_t launch_phys_tile_cn(const DevGraph &g, const DevState &st, const PhysTile &pt, int it, bool syn_only,
                               hipStream_t s);
// active_count[it] += tiles that still have a running frame after VN(it)
hipError_t launch_phys_tile_vn(const DevGraph &g, const DevState &st, const PhysTile &pt, int it, int *active_count,
                               int max_iter, hipStream_t s);  // active_count [2 max_iter]: tiles, then frames
// Syndrome of the posterior of iteration it right after VN(it), from the VN's
// hard-decision bytes, and the exits it implies (conv = it): the frames that
// converge there skip CN(it+1); active_count[it] / [max_iter + it] recounted
hipError_t launch_phys_tile_early_exit(const DevGraph &g, const DevState &st, const PhysTile &pt, int it,
                                       int *active_count, int max_iter, hipStream_t s);
// Monte-Carlo compaction of the running frames into tiles < nt (the finished ones counted first)
hipError_t launch_phys_compact(const DevGraph &g, const DevState &st, const PhysTile &pt, int nt, int cap, int *pairs,
                               hipStream_t s);
hipError_t launch_phys_tile_final(const DevGraph &g, const DevState &st, const PhysTile &pt, int max_iter,
                                  hipStream_t s);
hipError_t launch_phys_tile_out(const DevGraph &g, const DevState &st, const PhysTile &pt, uint8_t *z, float *post,
                                hipStream_t s);
hipError_t launch_phys_tile_count(const DevGraph &g, const DevState &st, const PhysTile &pt,
                                  unsigned long long *ctr, hipStream_t s);

// --- Philox4x32-10 (Salmon et al., SC'11), shared by host tests and device ---
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

}  // namespace ldpc
