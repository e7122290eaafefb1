/*
 * igr.h - C-ABI of the MI355X (gfx950) inductive graph-convolution path.
 *
 * Drop-in boundary for the DGL operator API the reference sits on.
 * The reference binds, from Python:
 *     g = dgl.graph((column, row), num_nodes=n, device=dev)      model.py:103-105, 4183, 4194
 *     dgl.ops.gspmm(g, 'mul', 'sum', lhs_data=X, rhs_data=vals)  model.py:106, 4184, 4196, 4037
 *     dgl.ops.gspmm(g, 'copy_rhs', 'max'|'sum', None, alpha)     model.py:4270, 4273 (AttIGCN)
 *     AttIGCN.masked_mm (index_select x2 + mul + sum)             model.py:4246-4255
 *     rep[users], rep[n_users + pos/neg] (BPR gathers)            model.py:4048-4049
 * Every entry point below replaces one of those; the ctypes binding that
 * calls them is inductive-recommendation_amd/igr/_lib.py.
 *
 * Conventions
 *  - Plain pointers and sizes.  Device pointers are HIP device memory
 *    allocated by the CALLER (PyTorch); this library never allocates, frees
 *    or synchronises inside a device entry point (graph-capture safe).
 *  - `stream` is a hipStream_t passed as void*; work is enqueued on it.
 *  - Return 0 on success, a non-zero IGR_ERR_* code otherwise; the message
 *    is in igr_last_error() (thread-local).  No C++ exception crosses the ABI.
 *  - Graph convention as in the reference: rows = destination nodes (DGL
 *    dst = `row`), columns = source nodes (DGL src = `column`).  Edge data
 *    (`rhs`) is indexed by EDGE ID; edge id = CSR position unless the graph
 *    carries an `edge_id` permutation (multigraph built from unsorted COO).
 *  - fp32 throughout (the reference computes in float32).
 */
#ifndef IGR_H
#define IGR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IGR_OK 0
#define IGR_ERR_ARG 1
#define IGR_ERR_HIP 2
#define IGR_ERR_UNSUPPORTED 3
#define IGR_ERR_INTERNAL 4

/* A CSR graph resident in device memory plus its row schedule.
 * Built once per graph by the host functions below (the reference rebuilds
 * a dgl.graph on every call, model.py:4183/4194; the values may change per
 * step, the structure never does). */
typedef struct igr_csr {
    int64_t n_rows;             /* destination nodes                              */
    int64_t n_cols;             /* source nodes (rows of lhs)                     */
    int64_t nnz;
    const int64_t *row_ptr;     /* [n_rows + 1]                                   */
    const int32_t *col_idx;     /* [nnz], sorted within each row                  */
    const int64_t *edge_id;     /* [nnz] CSR position -> edge id, or NULL (=id)   */
    /* schedule (igr_plan_fill): rows with degree <= split_threshold are
     * processed one per lane-group, heaviest first; longer rows are cut into
     * chunks of chunk_edges edges whose partial sums are combined in order
     * (deterministic, no atomics). */
    int64_t n_order;
    const int32_t *order;       /* [n_order] row ids                              */
    int64_t n_split;
    const int32_t *split_row;   /* [n_split] row ids                              */
    const int64_t *split_ptr;   /* [n_split + 1] chunk ranges                     */
    int64_t n_chunks;
    const int32_t *chunk_row;   /* [n_chunks]                                     */
    const int64_t *chunk_beg;   /* [n_chunks] first CSR position of the chunk     */
    int64_t chunk_edges;
} igr_csr;

/* Fused row epilogue of a SpMM:
 *   y[r]   = row_scale[r] * (alpha * (A x)[r] + beta * add[r])
 *            (add, row_scale may be NULL)
 *   acc_mode 1: acc[r] = y[r] / acc_div
 *   acc_mode 2: acc[r] = (acc[r] + y[r]) / acc_div
 * It fuses the layer-mean of LightGCN/IGCN get_rep (model.py:108-109,
 * 4198-4199) and the "+ g/(L+1)" of its backward into the SpMM; row_scale
 * lets the backward pre-scale dx_0 by the feature graph's row scale, so the
 * transposed feature SpMM gathers no per-edge column scale.  row_mask /
 * col_mask restrict a layer to the rows a training step's loss can reach
 * and its backward to the source rows that carry gradient. */
typedef struct igr_epilogue {
    float alpha;
    float beta;
    const float *add;
    int64_t ld_add;
    float *acc;
    int64_t ld_acc;
    int32_t acc_mode;
    float acc_div;
    int32_t skip_y;             /* 1: do not store y                             */
    const float *row_scale;     /* [n_rows] or NULL: IGCN's feature row scale    */
                                /* moved onto the reverse SpMM's source rows     */
    const uint32_t *row_mask;   /* bitmap [ceil(n_rows/32)] or NULL: rows whose  */
                                /* bit is clear are skipped (y, acc untouched)   */
    const uint32_t *col_mask;   /* bitmap [ceil(n_cols/32)] or NULL: edges whose */
                                /* column bit is clear add nothing, x unread     */
} igr_epilogue;

/* ------------------------------------------------------------------ misc */
const char *igr_last_error(void);
int igr_version(void);
/* Device properties used by the host side (CU count, L2, arch name). */
int igr_device_info(int device, int *n_cu, int *l2_bytes, char *arch, int arch_len);

/* ------------------------------------------------------- host graph build
 * Host (CPU) functions on host memory; multi-threaded (n_threads <= 0: all).
 * They replace the reference's Python/scipy construction
 * (utils.py:33-50, model.py:89-98, model.py:4139-4175). */

/* COO -> CSR sorted by (row, col).  dedup=1 sums duplicate (row, col)
 * entries (scipy .tocsr() + torch .coalesce(), utils.py:38, 47-49); dedup=0
 * keeps every edge (DGL multigraph) and records edge_id.  Output arrays hold
 * `nnz` entries; *nnz_out receives the stored count.  val/edge_id nullable. */
int igr_csr_from_coo(int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *row,
                     const int64_t *col, const float *val, int32_t dedup, int64_t *row_ptr,
                     int32_t *col_idx, float *val_out, int64_t *edge_id, int64_t *nnz_out,
                     int32_t n_threads);

/* Transposed CSR (reverse graph for the gspmm backward, model.py:106, 4196):
 * t_row_ptr [n_cols+1], t_col_idx [nnz] (= source row), t_pos [nnz] = CSR
 * position in the forward graph of each transposed entry. */
int igr_csr_transpose(int64_t n_rows, int64_t n_cols, const int64_t *row_ptr,
                      const int32_t *col_idx, int64_t *t_row_ptr, int32_t *t_col_idx,
                      int64_t *t_pos, int32_t n_threads);

/* Row sums of a CSR's values (degree when the values are 1; exact in fp32
 * below 2^24).  val NULL means 1. */
int igr_csr_row_sums(int64_t n_rows, const int64_t *row_ptr, const float *val, float *out);

/* Symmetric normalisation values (model.py:91-96):
 *   out[p] = (dinv_row[r] * val[p]) * dinv_col[col[p]]
 * dinv_col = dinv_row for the square adjacency; distinct for a rectangular
 * user x item block of a sharded graph.  val NULL means 1. */
int igr_sym_norm_values(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                        const float *val, const float *dinv_row, const float *dinv_col, float *out);

/* Row schedule.  igr_plan_size returns the array sizes, igr_plan_fill fills
 * host arrays that the caller copies to the device and references from
 * igr_csr.  Short rows are ordered by degree, descending, inside windows of
 * `window` consecutive rows (0 = one global window); long rows are chunked and
 * ordered heaviest first. */
int igr_plan_size(int64_t n_rows, const int64_t *row_ptr, int64_t split_threshold,
                  int64_t chunk_edges, int64_t *n_order, int64_t *n_split, int64_t *n_chunks);
int igr_plan_fill(int64_t n_rows, const int64_t *row_ptr, int64_t split_threshold,
                  int64_t chunk_edges, int64_t window, int32_t *order, int32_t *split_row,
                  int64_t *split_ptr, int32_t *chunk_row, int64_t *chunk_beg);

/* Occurrences of each id: counts[b] = #{i : ids[i] == b}, b in [0, n_bins).
 * The degree pass of utils.py:42-50 (a duplicate pair counts twice, as scipy's
 * summed duplicates do in the row sum of model.py:90) over one slice of an
 * interaction stream: the ranks of a sharded graph each count a slice and add
 * the counts up.  An id outside [0, n_bins) is an error. */
int igr_count_ids(int64_t n, const int64_t *ids, int64_t n_bins, int64_t *counts, int32_t n_threads);

/* The pairs of an interaction stream whose key lies in [lo, hi), in stream
 * order: out_key = key - lo, out_other = other.  *n_out receives the count;
 * with out_key == out_other == NULL only the count is computed (call once to
 * size the arrays, once to fill them).  This is how a rank of a sharded graph
 * keeps its own user range of the training pairs (the reference holds the
 * whole list in one process, dataset.py:94-114). */
int igr_select_id_range(int64_t n, const int64_t *key, const int64_t *other, int64_t lo, int64_t hi,
                        int64_t *out_key, int64_t *out_other, int64_t *n_out, int32_t n_threads);

/* ------------------------------------------------------- device kernels */

/* gspmm(g, 'mul', 'sum', lhs_data=x, rhs_data=rhs) - CSR SpMM, fp32.
 * Replaces dgl.ops.gspmm at model.py:106, 4184, 4196, 4037 (and its
 * reverse-graph backward).  x: [n_cols, d] with leading dim ldx; rhs: edge
 * weights by edge id (NULL = 1); y: [n_rows, d] with leading dim ldy.
 * workspace: n_chunks * d floats (NULL allowed when n_chunks == 0).
 * epi may be NULL (plain y = A x). */
int igr_spmm_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx, const float *rhs,
                 float *y, int64_t ldy, const igr_epilogue *epi, float *workspace, void *stream);

/* igr_spmm_f32 without the `workspace` argument and without any allocation.
 * No counterpart in the reference: it exists for callers that cannot allocate
 * device memory (code under hipGraph capture, tight serving loops, harnesses
 * that forbid hipMalloc).  The partial rows of split rows (n_chunks * d floats)
 * live in a static device array of IGR_SPMM_NOALLOC_MAX_FLOATS floats (16 MiB),
 * held by every GPU the library runs on until the process ends; a graph whose
 * n_chunks * d exceeds it is rejected with IGR_ERR_ARG.  Same results as
 * igr_spmm_f32, bit for bit.  All calls on one GPU share that GPU's array:
 * calls that overlap on one GPU (two streams, two threads) race.  Nothing in
 * the array needs clearing between calls.  The first call on a device looks up
 * the array's address (make it outside a stream capture).  The device that owns
 * the output must be the current one (hipSetDevice): the array is per device, and
 * a call whose output lives on another GPU is rejected with IGR_ERR_ARG. */
#define IGR_SPMM_NOALLOC_MAX_FLOATS (4 << 20)
int igr_spmm_noalloc_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx, const float *rhs,
                         float *y, int64_t ldy, const igr_epilogue *epi, void *stream);

/* SpMM with row / column scaled weights and fused dropout:
 *   w(p) = (row_scale ? row_scale[r] : 1) * (col_scale ? col_scale[c] : 1)
 *   if keep < 1: w = floor(keep + U) ? w / keep : 0,
 *                U = uniform(seed, offset, key(forward row, forward column))
 * The IGCN feature graph's values are row-constant (row_sum[r]^e,
 * model.py:4127-4130), so its dropout SpMM (model.py:4016-4028, 4184) needs
 * no per-edge array. The mask is keyed by the edge's (row, column) in the
 * frame it was drawn for (the coalesced feature graph has one edge per
 * pair); transposed = 1 runs g as the reverse of that frame, so the backward
 * regenerates the forward's mask without an edge-id permutation.  Rows and
 * columns < 2^32 when keep < 1.  Same epilogue / workspace contract as
 * igr_spmm_f32.  offset_dev (nullable, device int64): the draw offset is
 * offset + *offset_dev, read on the device - a step counter kept in HBM, so a
 * captured hipGraph draws a fresh mask on every replay. */
int igr_spmm_scaled_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx, const float *row_scale,
                        const float *col_scale, float keep, uint64_t seed, uint64_t offset,
                        const int64_t *offset_dev, int32_t transposed,
                        float *y, int64_t ldy, const igr_epilogue *epi, float *workspace, void *stream);

/* Per-head SpMM: y[r, j*d:(j+1)*d] = sum_{p in row r} rhs[eid(p)*h + j] * x[col[p], j*d:(j+1)*d]
 * for every head j < h, rhs [nnz, h] by edge id.  The backward of the h-head
 * SDDMM (AttIGCN.masked_mm, model.py:4246-4255: d x_q = A_alpha x_k per head,
 * d x_k on the reverse graph) without a per-head copy of rhs.  One launch
 * per head; same workspace contract as igr_spmm_f32. */
int igr_spmm_heads_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx, const float *rhs,
                       float *y, int64_t ldy, float *workspace, void *stream);

/* Row-restricted SpMM and its transpose (training step: the loss reads the
 * representation only at the batch rows, model.py:4048-4049 / 4049-4051, so
 * the last layer of get_rep, model.py:4196 / 106, is needed only there and
 * the first layer of its backward only pushes from there).  rows: int64
 * [n_sel] row ids, repeats allowed; rhs: CSR-position values (NULL = 1;
 * graphs with an edge_id permutation are not supported); d in {32, 64, 128,
 * 256}; one workgroup per selected row, its lane groups striding the row.
 *   igr_spmm_rows_f32: out[i] = scale * (sum_{p in row rows[i]} rhs[p] x[col[p]]
 *                                        + add_g[rows[i]] + add_i[i])
 *                      (add_g / add_i optional; fixed-order LDS reduction,
 *                      deterministic)
 *   igr_spmm_push_f32: dst[col[p]] += scale * rhs[p] * src[i] for p in row
 *                      rows[i], and dst[rows[i]] += scale * src[i] when
 *                      self_add (float atomics; summation order not fixed) */
int igr_spmm_rows_f32(const igr_csr *g, int32_t d, const int64_t *rows, int64_t n_sel, const float *x, int64_t ldx,
                      const float *rhs, const float *add_g, int64_t ld_g, const float *add_i, int64_t ld_i,
                      float scale, float *out, int64_t ldo, void *stream);
int igr_spmm_push_f32(const igr_csr *g, int32_t d, const int64_t *rows, int64_t n_sel, const float *src, int64_t lds,
                      const float *rhs, float scale, int32_t self_add, float *dst, int64_t ldd, void *stream);

/* Stable sort of row ids, the first step of every fixed-order accumulation
 * below (the reference's index_put backward, trainer.py:553, run sequentially
 * adds the terms of a repeated row in the order they appear; so do these):
 *   keys[k] = (row << 32) | e, ascending, for the concatenation of up to three
 *   index arrays of n entries each: entry e = a * n + i has row = idx_a[i] +
 *   off_a (idx1 / idx2 nullable).  Rows must lie in [0, 2^32 - 1).
 * keys: igr_rowsort_size(total) uint64 (total = n * number of arrays); the
 * first `total` hold the result, the rest is scratch. */
int64_t igr_rowsort_size(int64_t total);
int igr_rowsort(int64_t n, const int64_t *idx0, int64_t off0, const int64_t *idx1, int64_t off1,
                const int64_t *idx2, int64_t off2, uint64_t *keys, void *stream);

/* The push without atomics (the training backward uses this one): mark the
 * selected rows, sum repeated rows' sources into one slot each, then every
 * output row gathers only from marked columns:
 *   igr_rowset_mark:  bits[r/32] |= 1 << r%32, and the same for h = r mod 2^19 in
 *                     filter (bits, filter zero on entry; bits: uint32[(n+31)/32],
 *                     filter: uint32[16384])
 *   igr_rowset_sum_f32: sorted = igr_rowsort(rows); for the first position k of
 *                     every distinct row r: slot[r] = k and agg[k] = the sum of
 *                     scale * src[i] over rows[i] = r, i ascending (slot:
 *                     int32[n], agg: [n_sel, d]; other rows of agg untouched)
 *   igr_spmm_pull_marked_f32: out[c] = scale * (sum_{p in row c, col[p] marked}
 *                     rhs[p] agg[slot[col[p]]] + self_add [c marked] agg[slot[c]])
 *                     (one lane group per row, fixed order: bitwise
 *                     reproducible).  Persistent 1024-thread workgroups
 *                     keep the 64 KB filter in LDS; only filter hits probe bits.
 *                     row_mask (or NULL = every row): rows c with their bit
 *                     clear are not computed and out[c] is left untouched
 *   igr_rowset_clear: zero the words of bits and filter holding the selected rows
 * On the reverse graph, out = A^T G (+ G): igr_spmm_push_f32's result. */
int igr_rowset_mark(int64_t n_sel, const int64_t *rows, uint32_t *bits, uint32_t *filter, void *stream);
/* bits |= every column of the selected rows, and the row ids themselves when
 * self_mark (square graph): the rows at which a batch's last layer reads the
 * layer below it (the row_mask of that layer and the col_mask of its reverse,
 * igr_epilogue; trainer.py:537, model.py:4048-4049).  bits: uint32[(n_cols+31)/32].
 * scratch: NULL (atomic bit marks) or uint8[n_cols] of zeros, 16-byte aligned
 * (byte marks packed into bits afterwards; left zero again).
 * igr_bitmap_set: bits |= {idx[i]}. */
int igr_rowset_mark_neighbors(const igr_csr *g, int64_t n_sel, const int64_t *rows, uint32_t *bits,
                              int32_t self_mark, uint8_t *scratch, void *stream);
int igr_bitmap_set(int64_t n, const int64_t *idx, uint32_t *bits, void *stream);
int igr_rowset_sum_f32(int64_t n_sel, int32_t d, const uint64_t *sorted, const float *src, int64_t lds,
                       float scale, int32_t *slot, float *agg, int64_t ld_agg, void *stream);
int igr_spmm_pull_marked_f32(const igr_csr *g, int32_t d, const uint32_t *bits, const uint32_t *filter,
                             const int32_t *slot, const float *agg, int64_t ld_agg, const float *rhs, float scale,
                             int32_t self_add, const uint32_t *row_mask, float *out, int64_t ldo, void *stream);
int igr_rowset_clear(int64_t n_sel, const int64_t *rows, uint32_t *bits, uint32_t *filter, void *stream);

/* Eval ranking (BasicTrainer.eval, trainer.py:146-182): scores of a user batch
 * against every item (igr_gemm_f32), the user's train (and for 'test' val)
 * items set to -inf, then the top k per user.
 *   igr_mask_scores_f32: scores[r * ld + cols[p]] = -inf, p in [row_ptr[r], row_ptr[r+1])
 *                        (row_ptr may point into a larger CSR: absolute offsets)
 *   igr_topk_f32: out_idx[r*k + s] / out_val[r*k + s] (out_val nullable) = the k
 *                 largest of scores[r, 0:n_cols], ordered by value descending,
 *                 ties by index ascending (deterministic); 1 <= k <= min(1024, n_cols);
 *                 one workgroup per row, radix select + LDS bitonic sort. */
int igr_mask_scores_f32(int64_t n_rows, const int64_t *row_ptr, const int32_t *cols, float *scores, int64_t ld,
                        void *stream);
int igr_topk_f32(int64_t n_rows, int64_t n_cols, const float *scores, int64_t ld, int32_t k, float *out_val,
                 int64_t *out_idx, void *stream);

/* The uniforms igr_spmm_scaled_f32 draws, per CSR position of g (out[nnz]):
 * the explicit-values form of the same mask (AttIGCN's per-edge dropout,
 * model.py:4016-4028, feeds them to igr_edge_dropout_f32; tests).  offset_dev
 * as in igr_spmm_scaled_f32. */
int igr_dropout_uniforms(const igr_csr *g, uint64_t seed, uint64_t offset, const int64_t *offset_dev,
                         int32_t transposed, float *out, void *stream);

/* igr_edge_dropout_f32 with those uniforms drawn in the same pass (no rand array):
 * out[e] = val[e] / (1 - p) where floor((1 - p) + U_e) is 1, else 0, e by edge id
 * (NGCF.dropout_sp_mat, model.py:4016-4028, as a value mask over the fixed CSR). */
int igr_edge_dropout_counter_f32(const igr_csr *g, const float *val, float p, uint64_t seed, uint64_t offset,
                                 const int64_t *offset_dev, int32_t transposed, float *out, void *stream);

/* u_dot_v SDDMM: out[eid(p), h] = <u[row_p, h, :], v[col_p, h, :]>.
 * AttIGCN.masked_mm (model.py:4246-4255) with u = x_q (dst rows),
 * v = x_k (src rows); with h = 1 it is also the gspmm rhs-gradient.
 * u: [n_rows, h*d] (ld_u), v: [n_cols, h*d] (ld_v), out: [nnz, h]. */
int igr_sddmm_dot_f32(const igr_csr *g, int32_t h, int32_t d, const float *u, int64_t ld_u,
                      const float *v, int64_t ld_v, float *out, void *stream);

/* The attention SDDMM with one source row serving every head:
 *   igr_sddmm_shared_f32:      out[eid(p), j] = <u[row_p, j, :], v[col_p, :]>
 *   igr_spmm_shared_heads_f32: y[r, j, :] = sum_{p in row r} rhs[eid(p), j] * x[col_p, :]
 *                              (the gradient of the former with respect to u)
 * u, y: [n_rows, h*d]; v, x: [n_cols, d]; out, rhs: [nnz, h] by edge id.
 * AttIGCN's score <x_q[r, j], W_k[j] E[c] + b_k[j]> (model.py:4246-4268) equals
 * <W_k[j]^T x_q[r, j], E[c]> plus a term constant over the edges of row r, which the
 * row softmax that follows (model.py:4270-4274) cancels: with W_k[j]^T folded into
 * the query projection, every edge gathers the d floats of E[c] instead of the
 * h*d floats of x_k[c], and x_k is never formed.  d in {32, 64, 128, 256}, h a
 * power of two, h*d <= 512; 16-byte aligned operands. */
int igr_sddmm_shared_f32(const igr_csr *g, int32_t h, int32_t d, const float *u, int64_t ld_u,
                         const float *v, int64_t ld_v, float *out, void *stream);
int igr_spmm_shared_heads_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                              const float *rhs, float *y, int64_t ldy, void *stream);
/* The same with a workspace for the partial sums of split rows (the graph's schedule cuts
 * rows longer than its threshold into chunks, one wave each; a hub row - an item most users
 * rated - is otherwise one wave's serial loop): igr_spmm_shared_heads_workspace_size bytes,
 * 16-byte aligned; NULL = every row by one wave, as igr_spmm_shared_heads_f32.  A row's
 * chunk partials are added in chunk order (deterministic). */
int64_t igr_spmm_shared_heads_workspace_size(const igr_csr *g, int32_t h, int32_t d);
int igr_spmm_shared_heads_ws_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                                 const float *rhs, float *y, int64_t ldy, float *workspace,
                                 int64_t workspace_bytes, void *stream);

/* gspmm(g, 'copy_rhs', 'sum'|'max', None, x): out[r, h] = reduce over edges
 * of row r of x[eid, h]; empty rows give 0 (model.py:4270, 4273).
 * reduce: 0 = sum, 1 = max. */
int igr_segment_reduce_f32(const igr_csr *g, int32_t h, const float *x, int32_t reduce,
                           float *out, void *stream);

/* AttIGCN edge softmax, model.py:4270-4275, fused:
 *   m = segmax(alpha); a = exp((alpha - m[row]) / sqrt_d / 10); s = segsum(a);
 *   w[eid] = mean_h a / s[row]
 * keep (nullable, [nnz] by edge id): edges with keep == 0 are treated as
 * absent (dropout_sp_mat removes them from the reference's graph) - they
 * enter neither max nor sum and get w = 0.
 * row_max / row_sum ([n_rows, h]) are saved for the backward. */
int igr_att_softmax_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep, float sqrt_d,
                        float *w, float *row_max, float *row_sum, void *stream);
/* Backward of igr_att_softmax_f32: dalpha[eid, h] from dw[eid]. */
int igr_att_softmax_bwd_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep,
                            float sqrt_d, const float *row_max, const float *row_sum, const float *dw,
                            float *dalpha, void *stream);
/* The two with a workspace (igr_att_softmax_workspace_size bytes; the backward uses half):
 * the rows the graph's schedule splits are then processed chunk by chunk, a wave per chunk
 * (per-chunk max and sum, a per-row combine in chunk order, per-chunk weights), so a hub
 * row of any length is spread over the chip; row_max and row_sum must be given.  NULL
 * workspace = a workgroup per split row, as the plain entry points.  Deterministic. */
int64_t igr_att_softmax_workspace_size(const igr_csr *g, int32_t h);
int igr_att_softmax_ws_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep, float sqrt_d,
                           float *w, float *row_max, float *row_sum, float *workspace, int64_t workspace_bytes,
                           void *stream);
int igr_att_softmax_bwd_ws_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep, float sqrt_d,
                               const float *row_max, const float *row_sum, const float *dw, float *dalpha,
                               float *workspace, int64_t workspace_bytes, void *stream);

/* NGCF.dropout_sp_mat (model.py:4016-4028) as a value mask over the fixed
 * CSR: out = floor((1-p) + rand) ? val / (1-p) : 0.  rand ~ U[0,1), [n]. */
int igr_edge_dropout_f32(int64_t n, const float *val, const float *rand, float p, float *out,
                         void *stream);

/* IGCN.update_feat_mat (model.py:4127-4130): out[p] = row_sum[row_p] ^ exponent,
 * exponent = (alpha - 1)/2 - 0.5 (= 1/sqrt for alpha = 1).  With row_ptr ==
 * NULL one value per row is written (out[r] = row_sum[r] ^ exponent). */
int igr_feat_values_f32(int64_t n_rows, const int64_t *row_ptr, const float *row_sum,
                        float exponent, float *out, void *stream);

/* Row gather: out[i, :] = src[idx[i] + offset, :]  (rep[users], rep[n_users + pos],
 * model.py:4048-4049; Embedding lookups trainer.py:544-546). */
int igr_gather_rows_f32(int64_t n, int32_t d, const int64_t *idx, int64_t offset,
                        const float *src, int64_t ld_src, float *out, int64_t ld_out, void *stream);
/* Row scatter-add (gather backward, index_put accumulate): dst[row_i, :] += src[i, :]
 * with sorted = igr_rowsort of the n row ids (offset included).  Deterministic:
 * one writer per distinct row, adding its terms for i ascending onto the value
 * dst holds - the order of a sequential index_put / index_add (trainer.py:553). */
int igr_scatter_add_rows_f32(int64_t n, int32_t d, const uint64_t *sorted, const float *src,
                             int64_t ld_src, float *dst, int64_t ld_dst, void *stream);

/* Fused BPR step terms (model.py:4046-4052 + trainer.py:536-540, 542-548):
 * for each sample b: u = t[off_u + users[b]], p = t[off_i + pos[b]], n = t[off_i + neg[b]]
 *   s_b = sum_k u_k (n_k - p_k) * (w ? w_k : 1)
 *   loss[b] = softplus(s_b);  l2[b] = |u|^2 + |p|^2 + |n|^2      (loss/l2 nullable)
 * and, if grad != NULL, accumulates  g_loss * dloss_b/dt + g_l2 * dl2_b/dt
 * into grad; if dw != NULL, g_loss * dloss_b/dw into dw.  No atomics: with
 * sorted = igr_rowsort(batch, users, off_u, pos, off_i, neg, off_i) every
 * table row's terms are added in entry order (users, then pos, then neg, each
 * by sample) by one writer; sorted == NULL asserts that the 3 * batch rows are
 * all distinct (e.g. a table of gathered batch rows).  dw is summed per
 * workgroup, then over the workgroups, in sample order.  The backward
 * (grad or dw given) needs workspace: igr_bpr_workspace_floats(batch, d) floats.
 * (g_loss = dL/dloss_b, e.g. 1/batch for a mean.)  g_loss_dev / g_l2_dev
 * (nullable device scalars) multiply g_loss / g_l2: an autograd backward
 * passes the incoming gradient without a device->host sync. */
int64_t igr_bpr_workspace_floats(int64_t batch, int32_t d);
int igr_bpr_fwd_bwd_f32(int64_t batch, int32_t d, const int64_t *users, const int64_t *pos,
                        const int64_t *neg, int64_t off_u, int64_t off_i, const float *t,
                        int64_t ld_t, const float *w, float *loss, float *l2, float g_loss,
                        float g_l2, const float *g_loss_dev, const float *g_l2_dev, float *grad,
                        int64_t ld_grad, float *dw, const uint64_t *sorted, float *workspace,
                        void *stream);

/* Dense fp32 GEMM on MFMA (v_mfma_f32_16x16x4_f32, exact fp32 products):
 *   C[m, n] = sum_k A(m, k) * B(k, n) + bias[n]
 * A(m, k) = a[m*lda + k] (trans_a = 0) or a[k*lda + m] (trans_a = 1);
 * B(k, n) = b[n*ldb + k] (trans_b = 0: nn.Linear weight [N, K]) or
 *           b[k*ldb + n] (trans_b = 1).  bias nullable.
 * The d x d / d x 4d projections of NGCF (model.py:4039) and AttIGCN
 * (model.py:4259, 4264), forward and backward.  Outputs with few 64 x 64
 * tiles and a long K (the weight gradients, K = node count) split K over
 * workgroups when `workspace` holds igr_gemm_workspace_size(m, n, k) bytes
 * (NULL / smaller: no split); the splits are summed in order (deterministic). */
int64_t igr_gemm_workspace_size(int64_t m, int64_t n, int64_t k);
int igr_gemm_f32(int64_t m, int64_t n, int64_t k, const float *a, int64_t lda, int32_t trans_a,
                 const float *b, int64_t ldb, int32_t trans_b, const float *bias, float *c,
                 int64_t ldc, void *workspace, int64_t ws_bytes, void *stream);

/* Weight and bias gradients of a Linear applied to every node (the backward of NGCF's
 * Linear(d, d), model.py:4039, and AttIGCN's Linear(d, 4d), model.py:4259, 4264, under
 * loss.backward(), trainer.py:553):
 *   dw[n, c] = sum_m dy[m, n] * x[m, c]   (n < n_out, c < k_in),   db[n] = sum_m dy[m, n]
 * streamed over the m node rows with the dW block held in MFMA accumulators; partial
 * blocks of row ranges go to `workspace` (igr_linear_wgrad_workspace_size bytes, 16-byte
 * aligned) and are added in range order (the same bits on every run).  db nullable.
 * Supported: k_in in {32, 64, 128}, n_out in {64, 128} or a multiple of 256, dy / x 16-byte
 * aligned with leading dimensions a multiple of 4; other shapes: igr_gemm_f32 (trans_a). */
int64_t igr_linear_wgrad_workspace_size(int64_t m, int32_t n_out, int32_t k_in);
int igr_linear_wgrad_f32(int64_t m, int32_t n_out, int32_t k_in, const float *dy, int64_t ld_dy, const float *x,
                         int64_t ld_x, float *dw, int64_t ld_dw, float *db, void *workspace, int64_t ws_bytes,
                         void *stream);

/* ------------------------------------------------------- training step */

/* Device-side BPR sampler (dataset.py:119-131 semantics):
 * for each b < batch: users[b] = active[uniform], pos[b] = uniform item of that
 * user's sorted training list items[row_ptr[u] .. row_ptr[u+1]), neg[b] =
 * uniform item not in that list (rejection, at most max_rounds redraws).
 * Counter-based RNG: the draw is a pure function of (seed, offset, b), so a
 * step is reproducible and needs no RNG state.  offset_dev (nullable): offset +
 * *offset_dev read on the device (hipGraph-captured steps). */
int igr_bpr_sample(int64_t batch, int64_t n_active, const int32_t *active, const int64_t *row_ptr,
                   const int32_t *items, int64_t n_items, uint64_t seed, uint64_t offset,
                   const int64_t *offset_dev, int32_t max_rounds, int64_t *users, int64_t *pos, int64_t *neg,
                   void *stream);

/* Fused Adam step (torch.optim.Adam semantics, amsgrad off; trainer.py:44-46,
 * 555): one pass over p, g, m, v.  `step` is the 1-based
 * step count after increment (bias corrections).  step_dev (nullable, device
 * int64): the step is step + *step_dev and the bias corrections are formed on
 * the device (hipGraph-captured steps). */
int igr_adam_f32(int64_t n, float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                 double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                 const int64_t *step_dev, void *stream);

/* out[0] = mean(a[0..n)), out[1] = mean(b[0..n)) (b nullable: out[1] untouched):
 * the means of the per-sample loss and squared-norm terms that
 * igr_bpr_fwd_bwd_f32 writes (F.softplus(...).mean(), l2_norm_sq.mean();
 * trainer.py:539-540, 548), in one launch and a fixed summation order. */
int igr_means_f32(int64_t n, const float *a, const float *b, float *out, void *stream);

/* The step's scalar loss, trainer.py:551-552 (424-425 without the aux term):
 *     reg_loss = l2_reg * l2 + aux_reg * aux_loss;  loss = bpr_loss + reg_loss
 * from three device scalars (l2 / aux nullable), each operation rounded on its own
 * as in the tensor expression; loss_sum (nullable) += loss * weight is the epoch's
 * running sum (trainer.py:557, losses.update(loss.item(), batch size), kept on
 * the device). */
int igr_loss_combine_f32(const float *bpr, const float *l2, const float *aux, float c_l2, float c_aux,
                         float weight, float *loss, float *loss_sum, void *stream);

/* The same update for up to IGR_ADAM_MAX_SLOTS small tensors in one launch (projection
 * weights, biases, feature weights: the optimizer's loop over parameters, trainer.py:44-46,
 * 555).  `slots` is a host array; each slot's `step` is its own 1-based step count (added to
 * *step_dev when given, as in igr_adam_f32).  Bit-identical to igr_adam_f32 per tensor. */
#define IGR_ADAM_MAX_SLOTS 16
typedef struct igr_adam_slot {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;
    int64_t step;
} igr_adam_slot;
int igr_adam_multi_f32(int32_t n_slots, const igr_adam_slot *slots, double lr, double beta1, double beta2,
                       double eps, double weight_decay, const int64_t *step_dev, void *stream);

/* *counter += value on the stream (one device int64: the step counter a
 * captured training step advances at its end). */
int igr_counter_add(int64_t *counter, int64_t value, void *stream);

/* One value per node: y[r] = sum_{p in row r} rhs[eid(p)] * x[col[p]] (rhs NULL = 1), x [n_cols],
 * y [n_rows].  The width-1 case of gspmm(g, 'mul', 'sum', x, rhs) (reference model.py:4335 for
 * IMCGAE's repeated blocks, which stay one scalar per node through every layer).  Uses the
 * graph's row schedule when it has one (hub rows take a workgroup each); fixed summation
 * order. */
int igr_spmv_f32(const igr_csr *g, const float *x, const float *rhs, float *y, void *stream);

/* NGCF layer tail (reference model.py:4040-4042, after the two Linear layers):
 *   r   = dropout(leaky_relu(a + b, slope))     keep: 0/1 per element ([n, d], NULL = no
 *                                               dropout), kept elements times keep_scale
 *   nrm = r / max(|r|_2, 1e-12) per row         (F.normalize, written with leading dim ldn,
 *                                               e.g. into a column block of the concatenation)
 * row_norm[n] receives the clamped row norms for the backward.  a, b: [n, d] with leading
 * dimensions lda, ldb; r: [n, d] contiguous; 0 < d <= 256. */
int igr_layer_tail_f32(int64_t n, int32_t d, const float *a, int64_t lda, const float *b, int64_t ldb,
                       const float *keep, float keep_scale, float slope, float *r, float *nrm, int64_t ldn,
                       float *row_norm, void *stream);
/* Its gradient (loss.backward(), reference trainer.py:426): dz = d loss / d (a + b) from
 * gn = d loss / d nrm and gr = d loss / d r (either may be NULL), with r and row_norm of the
 * forward.  dz: [n, d] contiguous; it is the gradient of both a and b. */
int igr_layer_tail_bwd_f32(int64_t n, int32_t d, const float *gn, int64_t ldgn, const float *gr, int64_t ldgr,
                           const float *r, const float *row_norm, const float *keep, float keep_scale,
                           float slope, float *dz, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* IGR_H */
