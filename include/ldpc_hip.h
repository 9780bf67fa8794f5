/*
 * ldpc_hip.h -- C ABI of libldpc_hip.so, the MI355X (gfx950) SPA decoder.
 *
 * This is the drop-in boundary for the reference's hot path
 * (python_ldpc_app/spa_decoder.py).  Plain C types only: pointers, sizes,
 * int32/int64/double, and an opaque hipStream_t passed as void*.  The Python
 * host (ldpc-simulator_amd/ldpc_amd/) binds it with ctypes; INTEGRATION.md
 * shows the binding a maintainer of the reference would add.
 *
 * Conventions
 *   - Every function returns 0 on success or a negative LDPC_E* code; the
 *     message of the last failure on the calling thread is ldpc_last_error().
 *   - Decoding failure is NOT an error: it is status 1 (Result.DATA_TRANSFER_NOT_OK),
 *     exactly as spa_decoder.py:253 returns it.
 *   - The caller owns every I/O buffer.  Without LDPC_F_DEVICE_PTRS the I/O
 *     pointers are host memory and the call returns after the results are
 *     copied back; with it they are device pointers on the decoder's GPU and
 *     the call is asynchronous on `stream`.
 *   - A graph is immutable after creation and may be shared read-only by
 *     several decoders/threads.  A decoder (device workspace) is used by one
 *     thread at a time, like the reference's SPA_Decoder instance (main.py:221).
 *   - Frames are independent; a batch is split into chunks of at most the
 *     decoder's capacity and each chunk runs all its iterations on the GPU.
 */
#ifndef LDPC_HIP_H
#define LDPC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_ABI_VERSION 5  /* 5: LDPC_F_TEST_ZERO + ldpc_rare_rows_read (4: profile kinds LDPC_K_NKINDS 11) */

/* error codes */
#define LDPC_OK 0
#define LDPC_EINVAL (-22)  /* bad argument / malformed matrix                   */
#define LDPC_ENOMEM (-12)  /* host or device allocation failed                  */
#define LDPC_EDEVICE (-5)  /* HIP runtime error (message in ldpc_last_error)    */
#define LDPC_ERANGE (-34)  /* size does not fit the decoder / 32-bit indexing   */

/* decode flags */
#define LDPC_F_NLLR 0x1u        /* normalized-LLR metric, spa_decoder.py:210-228  */
#define LDPC_F_DEVICE_PTRS 0x2u /* I/O pointers are device pointers, async        */
#define LDPC_F_STATIC 0x4u      /* ldpc_mc_run: chunked schedule, no slot refill  */
#define LDPC_F_PHYS_HBM 0x8u    /* physical mode: HBM-resident state even if LDS fits */
#define LDPC_F_SPLIT 0x10u      /* parity decoder: separate CN/VN launches per iteration even
                                   where the tile-resident decoder applies (A/B, tests) */
#define LDPC_F_TEST_ZERO 0x20u  /* TEST ONLY (ldpc_generate_frames, ldpc_mc_run): frames whose global
                                   index F has F % 4 == 1 get a channel LLR of exactly 0.0 on identity
                                   column k + (131 F + 7) mod m and information column (37 F + 3) mod k,
                                   so their rows take spa_decoder.py:159-164's |t| <= 1e-10 branch (an
                                   identity column's M = (0 + E) - E is 0 on every iteration) */

typedef struct ldpc_hstd ldpc_hstd;       /* standard-form parity-check matrix  */
typedef struct ldpc_graph ldpc_graph;     /* H_std uploaded to one GPU          */
typedef struct ldpc_decoder ldpc_decoder; /* device workspace for one stream    */

/* ---------------------------------------------------------------- misc */
const char *ldpc_last_error(void);
int ldpc_abi_version(void);
/* number of visible GPUs (0 when none; never fails) */
int ldpc_device_count(void);

/* --------------------------------------------------- graph provider (host)
 * Replaces EncoderDecoderData.create_standart_parity_check_matrix
 * (encoder_decoder_data.py:269-317) and gaussian_elimination (:13-183):
 * GF(2) Gauss-Jordan with the same pivot rule (first row >= cur_row with a 1,
 * columns scanned 0..n-1), back-elimination, rank-deficient row drop (:280-305)
 * and the column permutation [non-pivot cols ascending] + [pivot cols in pivot
 * order] (:307-315).  Input: H (as read from the ALIST file, utils.py:21-113)
 * in CSR, 0-based, any column order within a row; duplicate (row,col) entries
 * are rejected with LDPC_EINVAL.
 */
int ldpc_hstd_build(int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                    ldpc_hstd **out);
/* Borrowed views valid until ldpc_hstd_free.  m_std = rank (rows kept). */
int ldpc_hstd_get(const ldpc_hstd *h, int32_t *m_std, int32_t *n, int64_t *nnz,
                  const int32_t **row_ptr, const int32_t **col_idx, const int32_t **perm);
void ldpc_hstd_free(ldpc_hstd *h);

/* ------------------------------------------------------------ graph (GPU)
 * Replaces SPA_Decoder.__init__ (spa_decoder.py:16-42): binds H_std (CSR,
 * ascending columns in every row -- the reference's check_to_var order) and
 * builds the column view (var_to_check, rows ascending) on the device of the
 * calling thread's current HIP device (`device` >= 0 selects one explicitly).
 * k = n - m information bits sit in columns 0..k-1 (H_std = [A | I_m]).
 */
int ldpc_graph_create(int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                      int32_t device, ldpc_graph **out);
int ldpc_graph_destroy(ldpc_graph *g);
/* Name of the check-node kernel the split parity path launches for this graph
 * on large batches ("cn_row_kernel": rows of degree <= 192 kept in registers,
 * 16 B/edge; "cn_kernel": one wavefront per row, 24 B/edge) -- measurement
 * labels.  Batches of <= 128 tiles of the 2304 codes (the streaming tail,
 * small split batches) run "cn_sub_kernel" instead (16-frame sub-tiles, t in
 * registers, 16 B/edge); the LDPC_K_CN profile kind counts whichever ran. */
const char *ldpc_cn_kernel_name(const ldpc_graph *g);
/* LDS bytes per workgroup of the tile-resident decoder for this graph, or 0 if
 * it does not apply.  It needs H_std = [A | I_m] and the A column sums of the
 * workgroup's frames in LDS: 64 frames (tile_kernels.hip: k*512 B + ~13 KB <=
 * 160 KB, row degree <= 192, e.g. wimax_576_0.5), else 16 or 8 frames
 * (tile_sub.hip: the WiMAX 2304 codes).  Where it applies, ldpc_decode_f64 and
 * the static schedule of ldpc_mc_run decode a whole chunk in ONE launch; the
 * separate per-iteration launches remain available via LDPC_F_SPLIT. */
int64_t ldpc_tile_lds_bytes(const ldpc_graph *g);
/* The tile-resident decoder this graph runs -- "tile_kernel" (64 frames per
 * workgroup), "tile_sub_kernel" (16 frames: wimax_2304_0.5) or "tile8_kernel"
 * (8 frames: the r3/4 codes, or any 2304 code whose graph was created with
 * LDPC_TILE8=1) -- or "" when it does not apply; measurement label. */
const char *ldpc_tile_kernel_name(const ldpc_graph *g);
/* Physical-mode kernel for this (sparse) graph: "phys_reg_kernel" / "phys_kernel"
 * (state in LDS) or "phys_cn_tile_kernel" (state in HBM). */
const char *ldpc_phys_kernel_name(const ldpc_graph *g, uint32_t flags);
int ldpc_graph_info(const ldpc_graph *g, int32_t *m, int32_t *n, int64_t *nnz,
                    int32_t *max_row_deg, int32_t *max_col_deg);

/* ---------------------------------------------------------- decoder
 * Device workspace for chunks of up to `max_frames` frames (rounded up to a
 * multiple of 64): fp64 messages E[tile][edge][64 frames], posteriors and
 * channel LLRs [tile][col][64], per-frame state.  Bytes needed:
 * ldpc_decoder_bytes().
 */
int64_t ldpc_decoder_bytes(const ldpc_graph *g, int32_t max_frames);
int ldpc_decoder_create(const ldpc_graph *g, int32_t max_frames, ldpc_decoder **out);
int ldpc_decoder_destroy(ldpc_decoder *d);
int32_t ldpc_decoder_capacity(const ldpc_decoder *d);

/*
 * Batched SPA decode, fp64, results equal to spa_decoder.py:63-280 per frame.
 * Replaces SPA_Decoder.decode(data_buffer) for `batch` frames at once.
 *   llr          [batch][n]  channel LLRs in H_std column order (data_buffer._channel_data)
 *   max_iter     >= 1        settings.get_max_iterations()
 *   z_out        [batch][n]  hard output z (= data_buffer._decoded_data), uint8, or NULL
 *   conv_out     [batch]     convergence_iteration (-1 if not converged) or NULL
 *   status_out   [batch]     0 = Result.OK, 1 = Result.DATA_TRANSFER_NOT_OK, or NULL
 *   post_out     [batch][n]  final a-posteriori LLRs, or NULL
 *   nllr_out     [batch]     _d_summarize_normalized_llr (needs LDPC_F_NLLR), or NULL
 *   nllr_hist    [batch][max_iter] per-iteration normalized LLR
 *                            (_normalized_llr_by_iterations; unused tail = -1), or NULL
 *   iters_out    [batch]     iterations executed (conv+1, or max_iter), or NULL
 *   msg_out      [batch][nnz] final check->variable messages E in H_std CSR
 *                            edge order (debug/parity; host memory only), or NULL
 *   stream       hipStream_t or NULL (null stream)
 */
int ldpc_decode_f64(ldpc_decoder *d, int32_t batch, const double *llr, int32_t max_iter,
                    uint32_t flags, uint8_t *z_out, int32_t *conv_out, int32_t *status_out,
                    double *post_out, double *nllr_out, double *nllr_hist, int32_t *iters_out,
                    double *msg_out, void *stream);

/* ------------------------------------------- on-device Monte-Carlo frames
 * Synthetic frame source that replaces DataBuffer(k) + encode + Channel
 * mode 1 (data_buffer.py:16-82, channel.py:38-81, generator.py:7-9) on the GPU:
 *   u  ~ iid bits from Philox4x32-10, key (seed), counter (frame, snr_point, block, 0)
 *   c  = [u, A.u mod 2]  (H_std = [A | I_m]), or for an IRA graph
 *        H = [H_info | staircase]: c = [u, p], p_r = p_{r-1} ^ (H_info u)_r
 *   x  = BPSK, bit 0 -> -1, bit 1 -> +1          (channel.py:49)
 *   y  = x + sigma^2 * g,  g ~ N(0,1) Box-Muller  (channel.py:68-76: noise std is sigma^2)
 *   llr = 2 y / sigma^2                           (channel.py:80)
 * sigma = 1/sqrt(2*speed*10^(snr/10)) is computed by the caller (channel.py:113).
 * ldpc_generate_frames writes them to host/device arrays (testing);
 * ldpc_mc_run generates, decodes and reduces counters without leaving the GPU.
 */
int ldpc_generate_frames(ldpc_decoder *d, uint64_t seed, int32_t snr_point, double sigma,
                         int64_t frame0, int32_t count, uint32_t flags, uint8_t *u_out,
                         double *llr_out, void *stream);

/* Counter vector per SNR point, int64[LDPC_MC_NCOUNT] (main.py:130-175 semantics):
 *   [0] frames  [1] failed (Result != OK)  [2] error bits in failed frames' info part
 *   [3] sum of convergence_iteration over converged frames  [4] converged frames
 *   [5] sum over frames of the final normalized-LLR count (nllr = count/k)
 *   [6] iterations executed (for roofline byte accounting)
 * Schedule: by default the decoder's max_frames are slots that are refilled
 * with the next frame index as soon as their frame stops (syndrome zero or
 * max_iter), so throughput follows the average iteration count rather than
 * the slowest frame of a tile; LDPC_F_STATIC decodes chunks of max_frames to
 * completion instead.  Both decode the same frames: counters are identical.
 */
#define LDPC_MC_NCOUNT 7
/* The streaming schedule's supply order of one point (ABI 4): the point's
 * local frame indices 0..count-1 (global frame0 + i) sorted by descending
 * syndrome weight of the channel hard decisions (llr > 0) on H_std, ties in
 * index order -- longest job first; order_out [count] int32, host memory.
 * ldpc_mc_run streams frames in this order unless LDPC_LPT=0 (the counters
 * are order-independent sums). */
int ldpc_frame_order(ldpc_decoder *d, uint64_t seed, int32_t snr_point, double sigma, int64_t frame0,
                     int32_t count, int32_t *order_out, void *stream);
int ldpc_mc_run(ldpc_decoder *d, uint64_t seed, int32_t n_points, const double *sigmas,
                int64_t frames_per_point, int64_t frame0, int32_t max_iter, uint32_t flags,
                int64_t *counters_out, void *stream);

/* ------------------------------------------------- physical mode (§8 f4)
 * NOT the reference's arithmetic.  Standard sum-product on a SPARSE graph --
 * pass H[:, perm] (the ALIST matrix in H_std column order, same code) to
 * ldpc_graph_create -- with the sign convention made consistent with the tanh
 * rule (Lambda = -llr), fp32.  A frame's state lives in LDS (one workgroup per
 * frame) when it fits (ldpc_phys_lds_bytes <= ~159 KB), otherwise -- or with
 * LDPC_F_PHYS_HBM -- in HBM, 64 frames per tile (csrc/phys_tile.hip); both
 * paths compute bit-identical results.  Inputs/outputs keep the reference's
 * conventions: llr as produced by channel.py, z = (bit estimate) ^ 1,
 * status 0 = OK.  The HBM path of ldpc_phys_decode synchronises before it
 * returns (it uses a temporary workspace), also with LDPC_F_DEVICE_PTRS.
 */
int64_t ldpc_phys_lds_bytes(const ldpc_graph *g);
int ldpc_phys_decode(const ldpc_graph *g, int32_t batch, const double *llr, int32_t max_iter, uint32_t flags,
                     uint8_t *z_out, int32_t *conv_out, int32_t *status_out, int32_t *iters_out, float *post_out,
                     void *stream);
/* On-device frames decoded in physical mode on g_phys; counters as
 * ldpc_mc_run (slot [5] unused).  The frame source is d_std's graph: either
 * the code's H_std = [A|I] (same generator as ldpc_mc_run), or -- for an IRA
 * code H = [H_info | staircase] such as the DVB-S2-profile code -- g_phys
 * itself (d_std created on g_phys; parities by accumulation).  On the HBM
 * path the running frames of a chunk are compacted into its first tiles once
 * at most a quarter of the slots still run (the finished frames counted
 * first): the counters are those of the uncompacted decode. */
int ldpc_phys_mc_run(ldpc_decoder *d_std, const ldpc_graph *g_phys, uint64_t seed, int32_t n_points,
                     const double *sigmas, int64_t frames_per_point, int64_t frame0, int32_t max_iter,
                     uint32_t flags, int64_t *counters_out, void *stream);

/* ------------------------------------------------------------ profiling
 * HIP-event timing of the decoder's own launches, on the stream they are
 * launched on (used by bench.py for the live roofline).  While enabled, every
 * kernel launch of this decoder is bracketed by events; ldpc_profile_read
 * synchronises, returns the summed milliseconds and launch counts per kind
 * (LDPC_K_*), and resets the accumulators.
 */
#define LDPC_K_CN 0      /* cn_kernel / cn_row_kernel / cn_sub_kernel (+ cn_rare_kernel): the split path's CN */
#define LDPC_K_VN 1      /* vn_kernel: the split path's per-tile VN */
#define LDPC_K_GEN 2
#define LDPC_K_COUNT 3
#define LDPC_K_PHYS 4
#define LDPC_K_PHYS_CN 5
#define LDPC_K_PHYS_VN 6
#define LDPC_K_TILE 7 /* tile-resident decoder: all iterations of a chunk (or a streamed SNR point) */
#define LDPC_K_CN_EDGE 8  /* few-frame path: cn_edge_kernel (lanes over a row's edges) */
#define LDPC_K_VN_EDGE 9  /* few-frame path: vn_edge_kernel + syn_kernel + tail_exit_kernel */
#define LDPC_K_VN_COLS 10 /* column-parallel VN: vn_cols_kernel + tail_exit_kernel (small batches,
                             streaming tail) */
#define LDPC_K_NKINDS 11
int ldpc_profile_enable(ldpc_decoder *d, int enable);
int ldpc_profile_read(ldpc_decoder *d, double *ms_out, int64_t *launches_out);
/* Rare rows (some |t| <= 1e-10, spa_decoder.py:159-164) this decoder has taken
 * since the last call, then reset (synchronises the device): out[0] = rows
 * queued to the split path's cn_rare_kernel (one per tile/row and iteration),
 * out[1] = rare rows the tile-resident decoders took in-kernel (one per
 * workgroup, row and pass).  A test hook: which code path saw the branch. */
int ldpc_rare_rows_read(ldpc_decoder *d, int64_t *out);

/* ------------------------------------------------ multi-GPU (RCCL, xGMI)
 * One process per GPU; frames are sharded by global index, so the only
 * exchange is ONE all-reduce of the int64 counter matrix per Monte-Carlo step
 * -- the reference's additive parent reduction of its workers' per-block
 * results (main.py:149-175).  librccl.so.1 (ROCm) is loaded on first use with
 * dlopen, so single-GPU users never load it.  No PyTorch.
 *   1. rank 0: ldpc_comm_unique_id(id); hand the 128 bytes to every rank
 *      (bench.py / ldpc_amd.comm: a file rendezvous on one node);
 *   2. every rank: ldpc_comm_init(id, rank, world, device, &c);
 *   3. ldpc_comm_allreduce(c, buf, count, dtype, op, flags, stream): in place;
 *      host buffers unless LDPC_F_DEVICE_PTRS (then async on `stream`);
 *      host buffers: synchronous.  dtype LDPC_DT_*, op LDPC_OP_*;
 *   4. ldpc_comm_barrier(c): all ranks arrive, then the device is synchronised;
 *   5. ldpc_comm_destroy(c).
 */
#define LDPC_COMM_ID_BYTES 128
#define LDPC_DT_I64 0
#define LDPC_DT_F64 1
#define LDPC_OP_SUM 0
#define LDPC_OP_MAX 1
typedef struct ldpc_comm ldpc_comm;
int ldpc_comm_unique_id(uint8_t *id_out);
int ldpc_comm_init(const uint8_t *id, int32_t rank, int32_t world, int32_t device, ldpc_comm **out);
int ldpc_comm_allreduce(ldpc_comm *c, void *buf, int64_t count, int32_t dtype, int32_t op, uint32_t flags,
                        void *stream);
int ldpc_comm_barrier(ldpc_comm *c);
int ldpc_comm_destroy(ldpc_comm *c);
/* hipDeviceSynchronize on `device` (bench.py's barrier brackets; no PyTorch) */
int ldpc_device_synchronize(int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_HIP_H */
