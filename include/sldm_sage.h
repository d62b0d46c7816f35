/*
 * sldm_sage.h — C ABI of the MI355X-native SageBlock hot path (libsldm_sage.so).
 *
 * The reference path is pure Python over PyTorch + torch_geometric 2.7.0 and has
 * no FFI of its own (there is no native code in the reference).  Each entry
 * point below replaces one step of what the reference executes per
 * SageBlock.forward (/root/reference/src/models/blocks/sageblock.py:16-20) and
 * its autograd backward; the replaced step is cited on each declaration.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer unless stated; the library allocates
 *     nothing: callers pass outputs and workspaces (the Python host code uses
 *     the PyTorch caching allocator);
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream); all
 *     work is enqueued asynchronously on it; no entry point synchronises;
 *   - matrices are row-major with a leading dimension in ELEMENTS;
 *   - dtype codes: SLDM_F32 (fp32) and SLDM_BF16 (bf16 storage, fp32 math);
 *   - return value: SLDM_OK or an error code; sldm_last_error() then returns a
 *     thread-local message.  Launch failures are reported from hipGetLastError.
 *   - thread safety: safe from any host thread; the only global state is the
 *     per-device address of sldm_gather_rows_split_static's scratch array
 *     (sldm_set_dropout_seed_source is per host thread);
 *   - HIP graph capture: every entry point only launches kernels on `stream`
 *     (no memset or copy nodes, no synchronisation), so a caller may record
 *     them into a graph -- with one exception: the radix sorts inside
 *     sldm_csr_build and sldm_degree_order switch, above 2^20 items, to a path
 *     that clears its histograms with memset nodes (build such graphs before
 *     the capture).  See sldm_set_dropout_seed_source for dropout.
 */
#ifndef SLDM_SAGE_H
#define SLDM_SAGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLDM_ABI_VERSION 9   /* 9: + sldm_set_dropout_seed_source; 8: + sldm_gemm_nt_rowscale_blocked(_ok) */

enum sldm_dtype { SLDM_F32 = 0, SLDM_BF16 = 1 };
enum sldm_status { SLDM_OK = 0, SLDM_ERR_ARG = 1, SLDM_ERR_HIP = 2 };

/* ABI version compiled into the library (== SLDM_ABI_VERSION). */
int sldm_abi_version(void);
/* Message of the last failed call on this host thread ("" if none). */
const char* sldm_last_error(void);

/* ---------------------------------------------------------------- graph ---
 * CSR build.  Replaces the per-call addressing of PyG
 * 2.7.0 MessagePassing.propagate (x.index_select(0, edge_index[0]) and the
 * scatter at edge_index[1]; called from sageblock.py:18) with, built once:
 *   rowptr[N+1], col[E]      CSR by destination: sources of node i's in-edges
 *   t_rowptr[N+1], t_col[E]  CSR by source (transpose): destinations
 * Within a row the entries keep the original edge order (stable), i.e. the
 * order in which PyG's CPU scatter_add_ accumulates.
 * edge_index is [2,E] (row 0 = source, row 1 = target), int64 if
 * index_is_int64 else int32.  Any id outside [0,N) sets *bad_index_flag
 * (device int32, caller-zeroed) to 1; outputs are then unspecified -- except
 * that an edge (N, N) is PADDING and is ignored (no counterpart in the
 * reference, where it would raise): a fixed-shape edge_index buffer, as a
 * captured HIP graph needs, fills its unused tail with it; rowptr[N] is then
 * the number of real edges and col / t_col hold them in front.
 * More than 2^20 edges: the sort inside records memset nodes, so such a build
 * must not be captured into a HIP graph (build it before the capture).
 * Requires N < 2^31 and E < 2^31.  t_rowptr/t_col may be NULL (forward only). */
size_t sldm_csr_workspace_bytes(int64_t num_edges, int64_t num_nodes);
int sldm_csr_build(const void* edge_index, int index_is_int64, int64_t num_edges,
                   int64_t num_nodes, int32_t* rowptr, int32_t* col,
                   int32_t* t_rowptr, int32_t* t_col, int32_t* bad_index_flag,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Longest-first row schedule for skewed (power-law) graphs: order[s] = the
 * row with the s-th largest rowptr degree (stable).  Gathering rows in this
 * order starts hub rows first and pairs rows of similar length in a wave;
 * results are unchanged (each row is still summed in CSR order). */
size_t sldm_degree_order_workspace_bytes(int64_t num_nodes);
int sldm_degree_order(const int32_t* rowptr, int64_t num_nodes, int32_t* order,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ----------------------------------------------------------- aggregation ---
 * out[i,:] = (addend[i,:] if addend) + S_i   with
 *   S_i = sum_{k in [rowptr[i], rowptr[i+1])} x[col[k], :]       (mean == 0)
 *   S_i = that sum / max(1, rowptr[i+1]-rowptr[i])               (mean == 1)
 * Sums are fp32, accumulated in CSR order (bit-identical to PyG's CPU
 * scatter_add_ for fp32 input).
 * Forward (mean=1, CSR by dst) replaces PyG 2.7.0 x.index_select(0, src) +
 * MeanAggregation / utils.scatter(reduce='mean').
 * Backward (mean=0, transpose CSR, x = inv_deg-prescaled dAgg, addend = the
 * lin_r input gradient) replaces autograd's gather + index_add_ (A8).
 * addend may be NULL; it has out's dtype.  row_order (nullable) is a row
 * schedule: slot s processes row row_order[s] (see sldm_degree_order). */
int sldm_gather_rows(int x_dtype, const void* x, int64_t ldx,
                     const int32_t* rowptr, const int32_t* col, const int32_t* row_order,
                     int64_t num_rows, int64_t feat, int mean,
                     const void* addend, int64_t ld_add,
                     int out_dtype, void* out, int64_t ldo, void* stream);

/* sldm_gather_rows with high-degree rows split (BASELINE C5: power-law
 * in-degrees up to ~10^4).  Rows with degree > max_deg
 * ("hubs", listed in hub_rows) are summed as fixed-length edge chunks:
 * chunk c covers CSR positions [chunk_beg[c], min(chunk_beg[c] + chunk_len,
 * rowptr[chunk_row[c]+1])) and is summed by its own row group into the fp32
 * row partials[c, 0:feat] (chunks of hub h are hub_chunk_ptr[h] ..
 * hub_chunk_ptr[h+1]-1, in CSR order); a second pass adds hub h's partials
 * in chunk order, then divides / adds the addend / stores like any row.
 * Every other row (all rows, or row_order's) is summed as in
 * sldm_gather_rows.  Deterministic; hub rows equal the CPU's sequential
 * order up to fp32 reassociation at chunk boundaries.  partials: num_chunks
 * x feat fp32 scratch.  Same dtype / addend / row_order contract as
 * sldm_gather_rows. */
int sldm_gather_rows_split(int x_dtype, const void* x, int64_t ldx,
                           const int32_t* rowptr, const int32_t* col, const int32_t* row_order,
                           int64_t num_rows, int64_t feat, int mean,
                           const void* addend, int64_t ld_add, int out_dtype, void* out,
                           int64_t ldo, const int32_t* hub_rows, const int32_t* hub_chunk_ptr,
                           int64_t num_hubs, const int32_t* chunk_row, const int32_t* chunk_beg,
                           int64_t num_chunks, int32_t chunk_len, int32_t max_deg,
                           float* partials, void* stream);

/* sldm_gather_rows_split without a workspace argument and without any device
 * allocation.  No counterpart in the reference: it exists for callers that
 * cannot allocate -- code under HIP graph capture, tight serving loops,
 * harnesses that forbid hipMalloc.  The chunk partials live in a static device
 * array inside the library (sldm_gather_rows_split_static_max_floats() floats
 * = 16 MiB, held by every GPU the library runs on until the process ends);
 * num_chunks * feat beyond that is rejected with SLDM_ERR_ARG.  The device
 * that is current at the call must be the stream's device.  All calls on one
 * GPU share the array: calls that overlap on one GPU (two streams, two host
 * threads) race; serialise them or use sldm_gather_rows_split.  Same results,
 * bit for bit, as sldm_gather_rows_split. */
size_t sldm_gather_rows_split_static_max_floats(void);
int sldm_gather_rows_split_static(int x_dtype, const void* x, int64_t ldx,
                                  const int32_t* rowptr, const int32_t* col,
                                  const int32_t* row_order, int64_t num_rows, int64_t feat,
                                  int mean, const void* addend, int64_t ld_add, int out_dtype,
                                  void* out, int64_t ldo, const int32_t* hub_rows,
                                  const int32_t* hub_chunk_ptr, int64_t num_hubs,
                                  const int32_t* chunk_row, const int32_t* chunk_beg,
                                  int64_t num_chunks, int32_t chunk_len, int32_t max_deg,
                                  void* stream);

/* g[i,:] = d[i,:] / max(1, rowptr[i+1]-rowptr[i]), in place, dtype of d.
 * Backward of the mean's division (A8) folded before the transpose sum. */
int sldm_scale_rows_by_inv_deg(int dtype, void* d, int64_t ld, const int32_t* rowptr,
                               int64_t num_rows, int64_t feat, void* stream);

/* ------------------------------------------------------------------ post ---
 * Forward of sageblock.py:11-13 fused with lin_l's bias (A6 epilogue, A7):
 *   hb   = h + bias                        (bias may be NULL)
 *   xhat = (hb - mean) * rstd,  rstd = 1/sqrt(var_biased + eps)
 *   y    = xhat * gamma + beta
 *   z    = y > 0 ? y : y * negative_slope  (ReLU: negative_slope = 0)
 *   out  = dropout(z)   keep iff u(seed, i*feat+j) >= drop_p, scale 1/(1-drop_p); drop_p in [0,1]
 * drop_p = 0 means Identity / eval mode.  xhat (out's dtype) and rstd (fp32)
 * are saved for the backward when non-NULL.  The dropout key of row i is
 * (seed, i + row_offset): a rank holding rows [r0, r1) of a partitioned graph
 * passes row_offset = r0 and draws the single-device mask. */
/* Dropout seeds of launches recorded into a HIP graph (nn.Dropout inside
 * sageblock.py:13 draws a new mask per call; a kernel argument is frozen at
 * capture).  While `device_word` is non-NULL, every launch this host thread
 * makes through an entry point that takes a `seed` keys its mask with
 * seed + *device_word (mod 2^64), the word read on the device when the kernel
 * runs: change the word between replays (a captured increment, or a copy from
 * the host) and each replay drops a different mask, the backward launches of
 * the same replay regenerating the forward's.  The word must stay allocated as
 * long as a graph holding such launches can run.  NULL (the initial state)
 * restores plain host seeds.  Per host thread; affects no launch already made. */
void sldm_set_dropout_seed_source(const uint64_t* device_word);

int sldm_post_fwd(int h_dtype, const void* h, int64_t ldh, int64_t num_rows, int64_t feat,
                  const float* bias, const float* gamma, const float* beta, float eps,
                  float negative_slope, float drop_p, uint64_t seed, int64_t row_offset,
                  int out_dtype, void* out, void* xhat, float* rstd, void* stream);

/* Backward of sldm_post_fwd (autograd of Dropout, LeakyReLU/ReLU, LayerNorm):
 *   dh = rstd * (g - mean_j(g) - xhat * mean_j(g*xhat)),  g = dy*gamma
 * col_partials[p, 0:F] += dy*xhat (dgamma), [p, F:2F] dy (dbeta),
 * [p, 2F:3F] dh (d bias of lin_l), over the rows handled by partial p
 * (num_partials in [1, 4096]); reduce with sldm_colsum.
 * zout (the forward output, nullable) decides the activation branch
 * (z > 0 <=> y > 0 exactly); without it y is recomputed from xhat. */
int sldm_post_bwd(int dtype, const void* dout, const void* xhat, const void* zout,
                  const float* rstd,
                  int64_t num_rows, int64_t feat, const float* gamma, const float* beta,
                  float negative_slope, float drop_p, uint64_t seed, int64_t row_offset,
                  int dh_dtype, void* dh, float* col_partials, int num_partials,
                  void* stream);
int sldm_post_num_partials(int64_t num_rows, int64_t feat);

/* out[j] = sum_p partials[p*width + j], fixed order (deterministic). */
int sldm_colsum(const float* partials, int num_partials, int64_t width, float* out,
                void* stream);

/* ----------------------------------------------------------- dense (MFMA) ---
 * Fused forward of one layer's dense part and post stack (A6 + A7):
 *   h   = [a0 | a1] · w^T + bias      a0 = agg [N,k0], a1 = x [N,k1],
 *                                     w = [W_l | W_r] as [nc, k0+k1] row-major
 *   out = dropout(act(LayerNorm(h)))  exactly as sldm_post_fwd
 * Replaces PyG SAGEConv's lin_l(agg) + lin_r(x) (sageblock.py:18) and
 * LayerNorm/act/Dropout (sageblock.py:11-13, :19).  nc <= 256.  xhat / rstd
 * may be NULL (no backward).  out and xhat are [N, nc] contiguous. */
int sldm_sage_dense_fwd(int dtype, const void* a0, int64_t lda0, int64_t k0,
                        const void* a1, int64_t lda1, int64_t k1, const void* w,
                        int64_t num_rows, int64_t nc, const float* bias,
                        const float* gamma, const float* beta, float eps,
                        float negative_slope, float drop_p, uint64_t seed, int64_t row_offset,
                        void* out, void* xhat, float* rstd, void* stream);

/* C[N, nc] = A[N, k] · B[nc, k]^T (both K-contiguous); columns j < scale_cols
 * are divided by max(1, rowptr[i+1]-rowptr[i]) when rowptr != NULL.
 * Backward of lin_l/lin_r w.r.t. their inputs (A8): A = dh, B = [W_l|W_r]^T,
 * giving [dAgg/deg | dx_root] in one pass.  With out2 != NULL the columns
 * j >= scale_cols go to out2[i, j - scale_cols] (ld ldo2) instead, so the
 * two halves land in separate contiguous [N, F_in] tensors: the transpose
 * gather then reads dAgg/deg rows from a table half the footprint of the
 * interleaved buffer (random-row gathers slow down with the table's span,
 * profiles/r1_gather_probe.txt).  out2 requires scale_cols % 4 == 0. */
int sldm_gemm_nt_rowscale(int dtype, const void* a, int64_t lda, int64_t k,
                          const void* b, int64_t ldb, int64_t num_rows, int64_t nc,
                          const int32_t* rowptr, int64_t scale_cols,
                          void* out, int64_t ldo, void* out2, int64_t ldo2, void* stream);

/* The same product with the degree-scaled half written column-blocked:
 * out_blocked is [scale_cols / blk_cols] blocks of [num_rows][blk_cols]
 * (block j = columns [j blk_cols, (j+1) blk_cols) of every row, contiguous),
 * the unscaled half goes to out2 [num_rows, nc - scale_cols] as above.  This
 * is the send layout of the all-to-all that turns a rank's row block into
 * every rank's column slice (feature-sliced partitions), written by the GEMM
 * instead of by a packing copy.  No reference counterpart (the reference has
 * no distributed code).  Shapes: ask sldm_gemm_nt_rowscale_blocked_ok (1 = the
 * call is supported; others return SLDM_ERR_ARG); values are bit-identical to
 * sldm_gemm_nt_rowscale's. */
int sldm_gemm_nt_rowscale_blocked_ok(int dtype, int64_t k, int64_t nc, int64_t scale_cols,
                                     int64_t blk_cols);
int sldm_gemm_nt_rowscale_blocked(int dtype, const void* a, int64_t lda, int64_t k,
                                  const void* b, int64_t ldb, int64_t num_rows, int64_t nc,
                                  const int32_t* rowptr, int64_t scale_cols,
                                  void* out_blocked, int64_t blk_cols, void* out2, int64_t ldo2,
                                  void* stream);

/* out[mo, n0+n1] (fp32) = sum_{r < num_rows} a[r, :]^T ⊗ [b0 | b1][r, :]
 * Weight gradients [dW_l | dW_r] = dh^T · [agg | x] (A8), split over the
 * node dimension into fp32 slabs summed in a fixed order (deterministic).
 * workspace: sldm_gemm_tn_workspace_bytes(num_rows, mo, n0+n1) bytes. */
size_t sldm_gemm_tn_workspace_bytes(int64_t num_rows, int64_t mo, int64_t nn);
int sldm_gemm_tn(int dtype, const void* a, int64_t lda, int64_t mo,
                 const void* b0, int64_t ldb0, int64_t n0,
                 const void* b1, int64_t ldb1, int64_t n1,
                 int64_t num_rows, float* out, void* workspace, size_t workspace_bytes,
                 void* stream);
/* The same product written as its two column blocks, out0[mo, n0] (= dW_l)
 * and out1[mo, n1] (= dW_r), each contiguous: the parameter gradients of
 * lin_l / lin_r (sageblock.py:8 SAGEConv, A8) without two slicing copies.
 * n0, n1 > 0; same workspace as sldm_gemm_tn; bit-identical values. */
int sldm_gemm_tn_split(int dtype, const void* a, int64_t lda, int64_t mo,
                       const void* b0, int64_t ldb0, int64_t n0,
                       const void* b1, int64_t ldb1, int64_t n1,
                       int64_t num_rows, float* out0, float* out1, void* workspace,
                       size_t workspace_bytes, void* stream);

/* Fused layer boundary of the backward: the transpose gather of layer l
 * (dx_l = addend + sum over out-edges of g, rows in row_order or 0..N-1)
 * rounded to the storage type and fed straight into layer l-1's
 * LayerNorm/activation/dropout backward (sldm_post_bwd's math, activation
 * branch from fma(xhat, gamma, beta)): writes dh (same dtype) and column
 * partials [num_partials][3][feat] for sldm_colsum.  Bit-identical dh to
 * sldm_gather_rows + sldm_post_bwd with zout = NULL; dx_l never reaches HBM.
 * Replaces the autograd of scatter_add_ / index_select (A8) of layer l and
 * of Dropout/act/LayerNorm (sageblock.py:11-13) of layer l-1. */
int sldm_gather_post_bwd_num_partials(int64_t num_rows, int64_t feat);
int sldm_gather_post_bwd(int dtype, const void* g, int64_t ldg, const int32_t* t_rowptr,
                         const int32_t* t_col, const int32_t* row_order, const void* addend,
                         int64_t lda, int64_t num_rows, int64_t feat, const void* xhat,
                         const float* rstd, const float* gamma, const float* beta,
                         float negative_slope, float drop_p, uint64_t seed, int64_t row_offset,
                         void* dh, float* col_partials, int num_partials, void* stream);

/* ------------------------------------------ multi-GPU layout switches ---
 * Feature-sliced SageBlock (sldm_sage/dist.py): rows [num_rows, B*bc] (row
 * stride ld_rows) <-> B column blocks [B][num_rows][bc] (contiguous), the
 * buffers the all-to-alls send / receive.  unpack optionally adds a
 * row-layout addend (dx = dx_root + gathered dAgg gradient, one rounding).
 * bc must be a multiple of 16 bytes' worth of elements. */
int sldm_cols_pack(int dtype, const void* rows_src, int64_t ld_rows, int64_t num_rows,
                   int64_t num_blocks, int64_t block_cols, void* blocks_dst, void* stream);
int sldm_cols_unpack(int dtype, const void* blocks_src, int64_t num_rows, int64_t num_blocks,
                     int64_t block_cols, const void* addend, int64_t ld_add, void* rows_dst,
                     int64_t ld_rows, void* stream);

/* ------------------------------------------------- graph-level readout ---
 * Global mean / max pooling over the batch vector:
 * replaces PyG 2.7.0 global_mean_pool / global_max_pool (grusage.py:3,
 * :119-127, :185), i.e. utils.scatter(x, batch, reduce='mean' | 'max') --
 * zeros(B,F).scatter_reduce_(0, batch, x, 'amax', include_self=False) on the
 * reference's CPU path.  The batch arrives as a segment CSR: seg_rowptr
 * [B+1] and member [N] (node ids, ascending within a segment; sldm_csr_build
 * of [arange(N); batch]).  Segments are processed in pieces of
 * sldm_segment_pool_piece_rows() rows: piece_ptr [B+1] is the prefix sum of
 * ceil(len_s / piece_rows) (num_pieces = piece_ptr[B]).
 * mean_out / max_out: [B, F] (either may be NULL); empty segments give 0.
 * max_divisor (fp32 [B, F], may be NULL): the number the upstream max
 * gradient is divided by -- members equal to the max, plus 1 when the max is
 * 0 (torch's amax backward also counts the zero-initialised self there).
 * max_first_row (int32 [B, F], may be NULL): the first member row holding
 * the max (x.max(dim) routing, PyG's batch=None global_max_pool). */
int sldm_segment_pool_piece_rows(void);
size_t sldm_segment_pool_workspace_bytes(int64_t num_pieces, int64_t feat);
int sldm_segment_pool(int dtype, const void* x, int64_t ldx, const int32_t* seg_rowptr,
                      const int32_t* member, int64_t num_segments, const int32_t* piece_ptr,
                      int64_t num_pieces, int64_t feat, void* mean_out, int64_t ld_mean,
                      void* max_out, int64_t ld_max, float* max_divisor,
                      int32_t* max_first_row, void* workspace, size_t workspace_bytes,
                      void* stream);

/* dx[i] = dmean[b]/count_b + (x[i] == max[b] ? dmax[b] / max_divisor[b] : 0),
 * b = seg_of[i] (int64, the batch vector); with max_first_row != NULL the max
 * term is instead dmax[b] at i == max_first_row[b] (x, max_out, max_divisor
 * unused).  dmean or dmax may be NULL. */
int sldm_segment_pool_bwd(int dtype, const void* x, int64_t ldx, const int64_t* seg_of,
                          const int32_t* seg_rowptr, int64_t num_nodes, int64_t feat,
                          const void* dmean, int64_t ld_dmean, const void* max_out,
                          int64_t ld_max, const void* dmax, int64_t ld_dmax,
                          const float* max_divisor, const int32_t* max_first_row, void* dx,
                          int64_t ld_dx, void* stream);

/* ------------------------------------------------ graph construction ---
 * Radius edges of a vehicle pack, replacing the
 * O(V^2 T) pair loop of gbuilder.py:85-111 / :241-268: for i, for j != i,
 * d = per-frame XY distance over the frames both vehicles are present in
 * (presence > 0.5); if any and min(d) <= radius: edge (i, j) with attr
 * [min, max, mean, mean of squares] -- numpy float32 arithmetic and order
 * reproduced exactly, edges i-major / j ascending.
 * pos: element strides (vehicle, frame, coordinate) of X (Y = X + sc);
 * presence: strides (vehicle, frame).  num_frames <= 256.
 * edge_index: int64 [2, capacity] (row 1 at + capacity), edge_attr fp32
 * [capacity, 4], capacity >= V(V-1); num_edges: device int32 (the edges
 * written, first num_edges columns). */
size_t sldm_radius_edges_workspace_bytes(int64_t num_vehicles);
int sldm_radius_edges(const float* pos, int64_t pos_sv, int64_t pos_st, int64_t pos_sc,
                      const float* presence, int64_t pres_sv, int64_t pres_st,
                      int64_t num_vehicles, int64_t num_frames, float radius,
                      int64_t* edge_index, int64_t capacity, float* edge_attr,
                      int32_t* num_edges, void* workspace, size_t workspace_bytes,
                      void* stream);

/* ------------------------------------------------------------ batching ---
 * Batch.from_data_list for the edge_index of G graphs resident on the device
 * (replaces PyG's collate behind main.py:166-167 for the
 * packs dataset.py:77 loads onto DEVICE), fused with the batch CSR pair:
 *   out_edge_index [2, out_ld] int64: graph g's edges at columns
 *     [E_<g, E_<g + E_g), ids + N_<g (PyG __inc__);
 *   out_batch [N] int64 (graph id per node), out_ptr [G+1] int64 (N_<g);
 *   rowptr/col (CSR by destination), t_rowptr/t_col (by source, nullable
 *   together), int32, rows in original edge order -- identical to
 *   sldm_csr_build on out_edge_index.
 * edge_index / edge_row_stride / num_edges / num_nodes are HOST arrays of G
 * entries (edge_index[g]: device pointer to int64 [2, stride], row 1 at
 * + stride).  bad_index_flag (device int32) is zeroed, then set to 1 if an id
 * lies outside [0, N_g) of its graph (those edges are left out of the CSR; the
 * caller raises).  N_g <= sldm_batch_graphs_max_nodes(). */
int sldm_batch_graphs_max_nodes(void);
int sldm_batch_graphs(int64_t num_graphs, const int64_t* const* edge_index,
                      const int64_t* edge_row_stride, const int64_t* num_edges,
                      const int64_t* num_nodes, int64_t* out_edge_index, int64_t out_ld,
                      int64_t* out_batch, int64_t* out_ptr, int32_t* rowptr, int32_t* col,
                      int32_t* t_rowptr, int32_t* t_col, int32_t* bad_index_flag, void* stream);

/* ------------------------------------------------------------------- GRU ---
 * The model's trajectory GRU: torch.nn.GRU(I -> H,
 * num_layers=1) as built at grusage.py:66-71 and called at :160-161
 * (gru_out, hlast = self.gru(x)), fp32, PyTorch's cell (aten RNN.cpp):
 *   r = s(x W_ir^T + b_ir + h W_hr^T + b_hr), z = s(... _iz ... _hz),
 *   n = tanh(x W_in^T + b_in + r (h W_hn^T + b_hn)), h' = (h - n) z + n.
 * x[n, t, i] at x + n*ldx_n + t*ldx_t + i (batch_first or time-major);
 * W_ih [3H, I], W_hh [3H, H] row-major in PyTorch's gate order (r, z, n);
 * biases and h0 [N, H] nullable (zeros).  out[n, t, :] = h_t (ldo_n, ldo_t),
 * h_n [N, H] nullable.  gates (nullable; needed by the backward):
 * sldm_gru_workspace_bytes(N, T, H) bytes.  Requires 1 <= I <= 16 and H a
 * multiple of 16 in [16, 96]. */
size_t sldm_gru_workspace_bytes(int64_t N, int64_t T, int64_t H);
int sldm_gru_fwd(const float* x, int64_t ldx_n, int64_t ldx_t, int64_t N, int64_t T, int64_t I,
                 int64_t H, const float* w_ih, const float* w_hh, const float* b_ih,
                 const float* b_hh, const float* h0, float* out, int64_t ldo_n, int64_t ldo_t,
                 float* h_n, float* gates, void* stream);

/* Backward of sldm_gru_fwd (autograd of nn.GRU): dout [N, T, H] (ldd_n, ldd_t)
 * and dh_n [N, H] are the upstream gradients (either nullable = zero); writes
 * dW_ih, dW_hh (overwritten, fp32), db_ih, db_hh (nullable), dh0 and dx
 * (nullable; dx at dx + n*lddx_n + t*lddx_t + i).  Weight gradients are summed
 * over per-workgroup partials in a fixed order (deterministic).
 * workspace: sldm_gru_bwd_workspace_bytes(N, T, I, H, dx != NULL). */
size_t sldm_gru_bwd_workspace_bytes(int64_t N, int64_t T, int64_t I, int64_t H, int need_dx);
int sldm_gru_bwd(const float* x, int64_t ldx_n, int64_t ldx_t, int64_t N, int64_t T, int64_t I,
                 int64_t H, const float* w_ih, const float* w_hh, const float* h0,
                 const float* out, int64_t ldo_n, int64_t ldo_t, const float* gates,
                 const float* dout, int64_t ldd_n, int64_t ldd_t, const float* dh_n, float* dx,
                 int64_t lddx_n, int64_t lddx_t, float* dh0, float* dw_ih, float* dw_hh,
                 float* db_ih, float* db_hh, void* workspace, size_t workspace_bytes,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SLDM_SAGE_H */
