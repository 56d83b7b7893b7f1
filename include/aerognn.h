/* aerognn.h — C-ABI of libaerognn.so, the MI355X (gfx950) hot path of the bi-stride
 * multi-scale MeshGraphNet (cudagu/aero-gnn).
 *
 * The reference is pure Python + PyTorch/torch_scatter: it has no FFI of its own.
 * Each entry point below replaces the aten / torch_scatter work that one reference Python
 * call performs; the Python mirror (aero-gnn_amd/models/) binds them with ctypes
 * (aero-gnn_amd/aerognn/_lib.py). Plain pointers and sizes only; every device pointer is
 * HBM memory owned by the caller; `stream` is a hipStream_t (NULL = default stream).
 * Return value: 0 on success, a hipError_t (>0) from the launch, or a negative AGN_E*
 * argument error (see agn_error_string).
 *
 * Replaces (reference file:line) --
 *   agn_mlp_forward   models/mlp.py:40-51 MLP.forward; models/mgnLayer.py:93-105 EdgeBlockSum
 *                     (+ gather of mgnLayer.py:103, residual :205); mgnLayer.py:32-49 EdgeBlock;
 *                     mgnLayer.py:134-153 NodeBlock incl. torch_scatter.scatter_add/mean (:144,146)
 *                     and the residual of :211
 *   agn_mlp_backward  autograd of the same
 *   agn_segment_sum   torch_scatter scatter_add/scatter_mean over a grouped (CSR/CSC) index:
 *                     mgnLayer.py:144-146 backward of index (:103), bsms_mgn.py:265,270,283
 *   agn_gather_rows   bsms_mgn.py:303-306 (_unpool_nodes) + :200 skip add; backward of
 *                     scatter_mean (gather / count)
 *   agn_radix_sort_*  bsms_mgn.py:242 torch.argsort(pos[:,0]) per graph (stable tie rule),
 *                     :280 torch.unique(keys) ordering; CSC/CSR construction for aggregation
 *   agn_pool_*        bsms_mgn.py:217-301 (_downsample: index map, coarse edge coalesce, means)
 *   agn_pack          layout conversion of nn.Linear weights into MFMA A-fragments
 *   agn_wgrad         weight / bias gradients of every Linear (mm(grad^T, input) in autograd)
 */
#ifndef AEROGNN_H
#define AEROGNN_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define AGN_MAX_LIN 8
#define AGN_MAX_SEG 3

enum { AGN_F32 = 0, AGN_BF16 = 1, AGN_F16 = 2, AGN_F64 = 3 };  /* F64: graph ops and the agn_f64_* entries */
enum { AGN_SEG_PLAIN = 0, AGN_SEG_GATHER = 1, AGN_SEG_SUM = 2, AGN_SEG_MEAN = 3 };
enum { AGN_E_ARG = -1, AGN_E_DTYPE = -2, AGN_E_HIDDEN = -3, AGN_E_SHAPE = -4 };
/* The MLP's hidden activation (mlp.py:37 getattr(F, activation_fn)): ReLU, GELU (exact erf form,
 * F.gelu's default), SiLU, tanh. For 16-bit storage the Linear output is rounded first and the
 * activation applied to the rounded value in fp32, then rounded (the bf16 module's order). */
enum { AGN_ACT_RELU = 0, AGN_ACT_GELU = 1, AGN_ACT_SILU = 2, AGN_ACT_TANH = 3 };

/* One input segment of a concatenated MLP input row (torch.cat in mgnLayer.py:44,151).
 * PLAIN : row r of ptr;  GATHER: row index[r] of ptr (x[row], x[col] of mgnLayer.py:40-41);
 * SUM/MEAN: sum (mean) of rows index[r] .. index[r+1]-1 of ptr (scatter_add / scatter_mean
 * of dst-grouped edges: index = CSC row pointer, rows grouped by receiver). */
typedef struct {
  int kind;
  int k;          /* features in this segment (<= hidden) */
  int ld;         /* row stride of ptr, elements */
  int _pad;
  const void* ptr;
  const int32_t* index;
  void* store;    /* optional: write the segment value (e.g. aggregated edges) [rows][k] */
} agn_seg;

typedef struct {
  int rows;
  int dtype;       /* activation storage dtype AGN_F32 / AGN_BF16 / AGN_F16 */
  int hidden;      /* 32, 64 or 128 */
  int nlin;        /* Linear layers in the chain (1..AGN_MAX_LIN), ReLU between */
  int out_dim;     /* features of the last Linear */
  int nseg;        /* input segments of layer 0 */
  int use_ln;      /* LayerNorm(out_dim) after the last Linear, eps 1e-5 */
  int out_ld;
  agn_seg seg[AGN_MAX_SEG];
  const void* wpk[AGN_MAX_LIN];    /* packed weights (agn_pack, trans = 0) */
  const float* bias[AGN_MAX_LIN];  /* fp32 bias or NULL */
  const float* ln_g;
  const float* ln_b;
  /* EdgeBlockSum prologue: layer-0 accumulator starts at P[src][0:H] + P[dst][H:2H] */
  const void* proj;                /* [*][2H] = [x W_s^T | x W_d^T + b] or NULL */
  const int32_t* src;
  const int32_t* dst;
  const void* resid;               /* y = resid + mlp(...) (row-major, ld = out_ld) or NULL */
  void* out;
  /* training saves (NULL when not needed) */
  void* act[AGN_MAX_LIN];          /* relu output of layer l (l < nlin-1), [rows][hidden], 16-B aligned */
  void* hpre;                      /* last Linear output before LN, [rows][out_dim] */
  float* stats;                    /* [rows][2] = mean, rstd */
  int tiled;                       /* 1: act/hpre in the tiled layout (AGN_TILED below, hidden-wide) */
  int act_fn;                      /* AGN_ACT_* between the Linears (0 = ReLU) */
  void* mask[AGN_MAX_LIN];         /* optional AGN_RELU_MASK of act[l] (may be given without act[l]; ReLU only) */
  void* pre[AGN_MAX_LIN];          /* optional (act_fn != ReLU, training): the rounded Linear output of
                                      hidden layer l before the activation, laid out as act[l] */
} agn_mlp_fwd_args;

typedef struct {
  int rows;
  int dtype;
  int hidden;
  int nlin;
  int out_dim;
  int in_dim;      /* K of layer 0 (sum of segment widths in forward) */
  int use_ln;
  int ln_rows;     /* out: rows of ln_partial written (<= agn_mlp_bwd_nwaves(rows)) */
  const void* wtpk[AGN_MAX_LIN];   /* packed TRANSPOSED weights (agn_pack, trans = 1) */
  const void* act[AGN_MAX_LIN];    /* not read (the ReLU backward uses mask[] below); kept for the layout */
  const void* hpre;
  const float* stats;
  const float* ln_g;
  /* upstream gradient of the MLP output (+ optional gathered add: g2[gidx[r]]);
   * g = NULL means a zero gradient (an output autograd left unused) */
  const void* g;
  const void* g2;
  const int32_t* gidx;
  /* outputs */
  void* gpre[AGN_MAX_LIN];         /* dL/d(pre-activation of layer l), [rows][M_l] */
  int din_nseg;                    /* segments of d(input of layer 0): widths din_k[s] */
  int din_k[AGN_MAX_SEG];
  void* din[AGN_MAX_SEG];          /* NULL = not needed */
  int din_resid[AGN_MAX_SEG];      /* 1: din[s] = g(+g2) + W0^T dh0 (residual of the block) */
  float* ln_partial;               /* [agn_mlp_bwd_nwaves(rows)][2][out_dim]: sum g*xhat, sum g */
  int tiled;                       /* 1: act/hpre are read in the tiled layout */
  int gpre_tiled;                  /* bit l: gpre[l] written in the tiled layout (hidden-wide only) */
  const void* mask[AGN_MAX_LIN];   /* AGN_RELU_MASK of hidden layer l < nlin-1 (required for ReLU) */
  int act_fn;                      /* AGN_ACT_* of the forward */
  int _pad3;
  const void* pre[AGN_MAX_LIN];    /* act_fn != ReLU: the forward's pre[l] (required), layout as act[l] */
} agn_mlp_bwd_args;

/* AGN_TILED layout of a [rows][H] activation saved for the backward (H = hidden, rows padded to
 * a multiple of 32): the 16-B register units of the 32-row wave that produced it, in register
 * order. Unit (row r, i, half h) lives at 16-B index ((r / 32) * U + i) * 64 + (r % 32) + 32 h,
 * U = (H / 2) * elem_size / 16 (units per lane half-row); for bf16 it holds features 16i+4h+{0..3} and 16i+8+4h+{0..3}, for fp32
 * features 8i+4h+{0..3}. One wave store/load instruction moves 1 KB contiguous. Only libaerognn
 * kernels read it (the MLP backward and agn_wgrad). */

/* AGN_RELU_MASK of a [rows][H] ReLU output (rows padded to 32): the sign bits the backward needs
 * instead of the activation. Per 32-row tile, ND = max(1, H / 64) dwords per lane of the producing
 * wave, dword (tile t, d, lane) at 4-B index (t * ND + d) * 64 + lane; bit j of dword d is
 * (activation register 32 d + j > 0) in the register order of AGN_TILED (register rho of lane
 * (row r % 32, half h) holds feature 8 (rho / 4) + 4 h + rho % 4). 16 B per row at H = 128
 * instead of 256 B. Only libaerognn kernels read it. */

/* Pack an A operand A[r][k] = trans ? W[k][r] : W[r][k] (r < rows, k < cols) into rows
 * [row_off, row_off+rows) x cols [col_off, col_off+cols) of a packed [dst_rows x dst_cols]
 * operand (row_off % 32 == 0, col_off % 16 == 0), so separate nn.Parameters (EdgeBlockSum's
 * src_lin / dst_lin, mgnLayer.py:122-129) pack into one concatenated operand. rows == 0:
 * copy a vector of `cols` values to fp32 at dst + col_off floats. */
typedef struct {
  const void* src;
  void* dst;
  int src_dtype;
  int dst_dtype;
  int rows;
  int cols;
  int trans;
  int ld;            /* row stride of W (elements) */
  int row_off;
  int col_off;
  int dst_rows;
  int dst_cols;
} agn_pack_desc;

/* ---- weight gradients: dW = G^T X, db = colsum(G) (autograd of every nn.Linear on the path:
 * mlp.py:42-46, mgnLayer.py:97-99 / :147-149, :127-132) ---- */
#define AGN_MAX_WGRAD 8
typedef struct {
  const void* g;        /* [rows][m] pre-activation grads (activation dtype) */
  const void* x;        /* [rows][k] layer input */
  int ldg, ldx;         /* row strides (elements) */
  int m, k, rows;
  int ldw;              /* row stride of dw (floats) */
  float* dw_partial;    /* agn_wgrad_partial_floats(m, k, nsplit) scratch */
  float* db_partial;    /* nsplit * round_up(m, 128) scratch, or NULL (no bias) */
  float* dw;            /* [m][ldw] fp32 output */
  float* db;            /* [m] fp32 output or NULL */
  int g_tiled, x_tiled; /* operand in the AGN_TILED layout (then m resp. k == 128) */
  int nsplit;           /* row splits of this desc (agn_wgrad_plan); dw_partial holds nsplit slabs */
  int _pad;
  const int32_t* xidx;  /* NULL, or a gathered X: logical row r is x's row xidx[r] (x[src] / x[dst]
                           of the concat edge MLP, mgnLayer.py:10-49, without an [E][k] copy);
                           row-major x only (x_tiled == 0) */
} agn_wgrad_desc;
typedef struct {
  int n;
  int _pad;
  agn_wgrad_desc d[AGN_MAX_WGRAD];
} agn_wgrad_batch;
int agn_wgrad_nsplit(int rows, int ndesc_blocks);
size_t agn_wgrad_partial_floats(int m, int k, int nsplit);
/* Fill d[i].nsplit: one wave of resident workgroups over the batch, the same split count for every
 * desc (agn_wgrad_nsplit of the largest). Host-only, no launch. */
int agn_wgrad_plan(agn_wgrad_batch* b);
/* nsplit > 0: every desc uses nsplit splits; nsplit <= 0: each desc uses its own d[i].nsplit */
int agn_wgrad(const agn_wgrad_batch* b, int dtype, int nsplit, void* stream);
/* out[c] = sum_r p[r][c] (r < nw, c < n) in fixed order via scratch[scratch_rows][n] */
int agn_colsum(const float* p, int nw, int n, float* scratch, int scratch_rows, float* out, void* stream);

int agn_version(void);
const char* agn_error_string(int code);
/* Process-wide kernel-selection options (testing / A-B measurement). Returns the previous value
 * or AGN_E_ARG. AGN_OPT_RESIDENT: 1 (default) = persistent resident-weight kernels for the
 * large bf16 H=128 edge MLPs, 0 = always the general kernels (bitwise-identical outputs).
 * (Keys 1-4 selected measured-slower edge-forward variants, removed in round 6; rejected.) */
enum {
  AGN_OPT_RESIDENT = 0
};
int agn_set_option(int key, int value);
/* bytes of a packed A operand with `m` rows and `k` reduction columns */
size_t agn_packed_bytes(int m, int k, int dtype);
/* max_threads >= max over descs of packed 16-B units (or vector length). src_dtype / dst_dtype must be
 * AGN_F32 / AGN_BF16 / AGN_F16; a descriptor with another dtype (it lives in device memory, so it
 * cannot be checked here without a copy) writes nothing. */
int agn_pack(const agn_pack_desc* descs_device, int n, int max_threads, void* stream);

int agn_mlp_forward(const agn_mlp_fwd_args* a, void* stream);
/* rows of ln_partial written by agn_mlp_backward (one per 256-row block) */
int agn_mlp_bwd_nwaves(int rows);
int agn_mlp_backward(const agn_mlp_bwd_args* a, void* stream);
/* out[c] = sum_w partial[w][c], c < n, fixed order (deterministic LN parameter grads) */
int agn_reduce_partials(const float* partial, int nw, int n, float* out, void* stream);

/* out[r] = sum (or mean) of src[perm ? perm[j] : j] for j in ptr[r]..ptr[r+1]-1; [rows][k] */
int agn_segment_sum(int rows, int k, int dtype, const int32_t* ptr, const int32_t* perm,
                    const void* src, int src_ld, void* out, int out_ld, int mean, void* stream);
/* out[r] = (base[r] + A[r]) + B[r], A[r] = sum_{j in ptr_a[r]..} src_a[perm_a ? perm_a[j] : j] and
 * B[r] likewise, each group summed from zero in index order, fp32, one rounding: the concat edge
 * MLP's node gradient dx + scatter_add(d x_src, src) + scatter_add(d x_dst, dst)
 * (mgnLayer.py:10-49 backward) in one pass. out may alias base; base NULL = 0. */
int agn_segment_sum2(int rows, int k, int dtype, const void* base, int base_ld, const int32_t* ptr_a,
                     const int32_t* perm_a, const void* src_a, int lda, const int32_t* ptr_b,
                     const int32_t* perm_b, const void* src_b, int ldb, void* out, int out_ld, void* stream);
/* Global max pooling (poolmgn.py:40, torch_geometric global_max_pool = scatter 'max'):
 * out[r][f] = max of src[perm ? perm[j] : j][f], j in ptr[r]..ptr[r+1]-1 (0 if empty), argmax[r][f]
 * = the first member row attaining it (-1 if empty); the backward writes dx[argmax[r][f]][f] =
 * gout[r][f] into a zero-filled dx. */
int agn_segment_max(int rows, int k, int dtype, const int32_t* ptr, const int32_t* perm, const void* src,
                    int src_ld, void* out, int out_ld, int32_t* argmax, void* stream);
int agn_segment_max_backward(int rows, int k, int dtype, const int32_t* argmax, const void* gout, int gout_ld,
                             void* dx, int dx_ld, void* stream);
/* out[r] = src[idx[r]] * (inv_count ? 1/max(cnt[idx[r]],1) : 1) + (add ? add[r] : 0) */
int agn_gather_rows(int rows, int k, int dtype, const int32_t* idx, const void* src, int src_ld,
                    const int32_t* cnt_ptr, const void* add, int add_ld, void* out, int out_ld,
                    void* stream);

/* Stable LSD radix sort of (key, value) pairs on `bits` low key bits. tmp buffers hold n each;
 * agn_radix_sort_temp_bytes gives the scratch size. Result ends in keys/vals. */
size_t agn_radix_sort_temp_bytes(int n);
int agn_radix_sort_u64(uint64_t* keys, int32_t* vals, int n, int bits, uint64_t* keys_tmp,
                       int32_t* vals_tmp, void* scratch, void* stream);
/* CSR row pointer of sorted int keys: ptr[v] = first i with key[i] >= v, v = 0..nrows */
int agn_row_ptr(const int32_t* sorted_keys, int n, int nrows, int32_t* ptr, void* stream);

/* exclusive prefix sum of n int32; *total (optional) = sum; scratch: agn_scan_temp_bytes(n) */
size_t agn_scan_temp_bytes(int n);
int agn_exclusive_scan_i32(const int32_t* in, int32_t* out, int n, int32_t* total, int32_t* scratch,
                           void* stream);
/* group_by's stable-sort input: keys[i] = keys32 ? keys32[i] : keys64[i] (as u64), vals[i] = i */
int agn_iota_keys(int n, const int32_t* keys32, const int64_t* keys64, int64_t* keys, int32_t* vals, void* stream);
/* CSC level of a reference edge_index [2][ld] int64 (mgnLayer.py:143-146 receivers `col`): given
 * perm (int32, edges stably grouped by receiver), src[i] = edge_index[0][perm[i]], dst[i] =
 * edge_index[1][perm[i]] (int32), perm64[i] = perm[i], inv64[perm[i]] = i (and inv32, if not NULL). */
int agn_level_index(int e, const int64_t* edge_index, int64_t ld, const int32_t* perm, int32_t* src, int32_t* dst,
                    int64_t* perm64, int64_t* inv64, int32_t* inv32, void* stream);
/* same as agn_row_ptr for sorted int64 keys (PyG `batch` vectors) */
int agn_row_ptr_i64(const int64_t* sorted_keys, int n, int nrows, int32_t* ptr, void* stream);

/* ---- bi-stride pooling (bsms_mgn.py:217-301) ----
 * 1. agn_pool_sort_keys + agn_radix_sort_u64: nodes ordered by (graph, x) — the per-graph
 *    argsort(pos[:,0]) of bsms_mgn.py:240-243 with the stable (x, node id) tie rule; pos == NULL
 *    keeps node order (bsms_mgn.py:244-245).
 * 2. agn_pool_assign: f2c = rank // stride + coarse offset of the graph (bsms_mgn.py:247-256),
 *    coarse members grouped per coarse node in ascending fine id (c2f, c2f_ptr), coarse batch.
 * 3. agn_pool_edge_candidates / _sort / _emit: coarse edge coalescing (bsms_mgn.py:276-288):
 *    per coarse receiver, the fine edges of its members sorted by (f2c[src], reference order)
 *    and run-length encoded -> coarse CSC (csrc, cdst), member ranges (cmem_ptr into cand_sorted),
 *    inverse map, and the coarse level's reference-order key (row * Nc + col). */
int agn_pool_sort_keys(int n, const int64_t* batch, const float* pos, int pos_ld, uint64_t* keys,
                       int32_t* vals, void* stream);
int agn_pool_assign(int n, int nc, int ngraph, const int64_t* batch, const int32_t* sorted_nodes,
                    const int32_t* gstart, const int32_t* coff, int stride, int32_t* f2c,
                    int32_t* c2f, int32_t* c2f_ptr, int64_t* cbatch, void* stream);
int agn_pool_edge_candidates(int nc, const int32_t* c2f, const int32_t* c2f_ptr, const int32_t* rowptr,
                             int32_t* cand_cnt, void* stream);
int agn_pool_edge_sort(int nc, const int32_t* c2f, const int32_t* c2f_ptr, const int32_t* rowptr,
                       const int32_t* src, const int64_t* refkey, const int32_t* f2c,
                       const int32_t* cand_ptr, int32_t* cand_tmp, int32_t* cand_sorted,
                       int32_t* uniq, void* stream);
int agn_pool_edge_emit(int nc, const int32_t* cand_ptr, const int32_t* cand_sorted,
                       const int32_t* src, const int32_t* f2c, const int32_t* crowptr,
                       int32_t* csrc, int32_t* cdst, int32_t* cmem_ptr, int32_t* inv,
                       int64_t* crefkey, int e_fine, void* stream);
/* ---------------------------------------------------------------------------------------
 * BSMS-GNN bi-stride operators (stale models/bistride_ops + old models/bsms_mgn, recovered
 * in SURVEY Appendix A; not reachable from the reference's train.py).
 *   agn_bfs_distance     BistridePooling.bfs_distance (bistride_ops @21): hop distances over the
 *                        out-adjacency (CSR rowptr/nbr of edge_index[0] -> [1]); -1 = unreachable.
 *                        work: agn_bfs_work_ints(n) int32. Synchronises the stream per 32 levels.
 *   agn_center_seed      argmin |pos - mean(pos)| (select_bistride_nodes @56, pos given)
 *   agn_maxdeg_seed      argmax bincount(edge_index[0]) (pos absent); first index on ties
 *   agn_bistride_select  where(dist even & >= 0), or where(dist >= 0) when that keeps < 30 %
 *                        (ascending); *nsel returned on the host (synchronises)
 *   agn_index_map        map[sel[j]] = j, -1 elsewhere (create_multiscale_graph @32)
 *   agn_subgraph_edges   keep edges with both ends selected, remap, drop self loops (order kept)
 *   agn_scatter_rows     out[idx[r]] = src[r] (Unpool.forward @102 after a zero fill)
 *   agn_wec_forward/backward  WeightedEdgeConv (bistride_ops @131-210), see agn_wec_args
 * ------------------------------------------------------------------------------------- */
size_t agn_bfs_work_ints(int n);
int agn_bfs_distance(const int32_t* rowptr, const int32_t* nbr, int n, int seed, int32_t* dist, int32_t* work,
                     int* levels_out, void* stream);
int agn_center_seed(const float* pos, int n, int pos_dim, int pos_ld, int32_t* seed, void* stream);
int agn_maxdeg_seed(const int32_t* rowptr, int n, int32_t* seed, void* stream);
size_t agn_compact_work_ints(int n);
int agn_bistride_select(const int32_t* dist, int n, int32_t* sel, int* nsel, int32_t* work, void* stream);
int agn_index_map(const int32_t* sel, int nsel, int n, int32_t* map, void* stream);
int agn_subgraph_edges(const int64_t* src, const int64_t* dst, int e, const int32_t* map, int64_t* osrc,
                       int64_t* odst, int* ecount, int32_t* work, void* stream);
int agn_scatter_rows(int rows, int k, int dtype, const int32_t* idx, const void* src, int src_ld, void* out,
                     int out_ld, void* stream);

/* WeightedEdgeConv: w_e = sigmoid(w2 . relu(W1 [x_src, x_dst, |pos_dst - pos_src|] + b1) + b2),
 * out_v = sum_{e: dst_e = v} (x T^T + b_T)[src_e] * w_e  ('mean': / max(deg_v, 1)).
 * The node projections pab = [x W1a^T | x W1b^T + b1] and tx = x T^T + b_T come from
 * agn_mlp_forward; edges are visited in the level's CSC order (sums in caller edge order). */
typedef struct {
  int n, e;
  int dtype;                 /* AGN_F32 / AGN_BF16 / AGN_F16 (x, pab, tx, weights, out, grads) */
  int out_dim;               /* 64 or 128 */
  int hid;                   /* edge-weight MLP hidden width: 64 */
  int pos_dim, pos_ld;       /* pos: fp32 [n][pos_ld], pos_dim <= 4 */
  int mean;                  /* 0 = 'add', 1 = 'mean' */
  const int32_t* rowptr;     /* CSC by receiver [n+1] */
  const int32_t* src;        /* [e] CSC order */
  const int32_t* dst;        /* [e] CSC order (backward) */
  const int64_t* perm;       /* [e] CSC position -> caller edge id */
  const int32_t* rowptr_src; /* CSR by sender [n+1] (backward) */
  const int32_t* perm_src;   /* [e] CSR entries -> CSC positions (backward) */
  const float* pos;
  const void* pab;           /* [n][2*hid] */
  const void* tx;            /* [n][out_dim] */
  const float* w1c;          /* [hid] weight column of the edge length */
  const float* w2;           /* [hid + 1] = second Linear's weight row | its bias b2 */
  const void* w_in;          /* [e] given weights (caller order) or NULL = compute them */
  void* w_out;               /* [e] computed weights (caller order) or NULL */
  void* out;                 /* [n][out_dim]; NULL = weights only (compute_edge_weights) */
  const void* dout;          /* backward: [n][out_dim] */
  const void* gw;            /* backward: grad of the returned weights [e] (caller order) or NULL */
  float* s_csc;              /* backward scratch: [e] weights in CSC order */
  float* dh;                 /* backward scratch: [e][hid] */
  void* dpa;                 /* backward out: [n][hid] */
  void* dpb;                 /* backward out: [n][hid] */
  void* dtx;                 /* backward out: [n][out_dim] */
  void* dw_in;               /* backward out: grad of the given weights [e] (caller order) or NULL */
  float* partial;            /* backward out: [agn_wec_blocks(n)][2*hid+1] = dw2 | dw1c | db2 partials */
} agn_wec_args;

int agn_wec_blocks(int n);
int agn_wec_forward(const agn_wec_args* a, void* stream);
int agn_wec_backward(const agn_wec_args* a, void* stream);

/* ---- fused training backward of the sum-trick edge MLP with forward recompute and in-kernel
 * weight gradients (bf16, H = 128; the EdgeBlockSum chain h0 = e W_e^T + P_s[src] + P_d[dst] ->
 * ReLU -> Lin1 -> ReLU -> Lin2 -> ReLU -> Lin3 -> LayerNorm, mgnLayer.py:72-105, and the residual
 * e' = e + ., mgnLayer.py:205). Replaces agn_mlp_backward + the chain's agn_wgrad share for that
 * chain, and lets the training forward save nothing: one persistent launch recomputes h0..h3
 * from e and the projection rows (bitwise the forward kernel's values), runs the LayerNorm
 * backward and the chain rule, and accumulates dW1..dW3 / db1..db3 on chip, so no activation and
 * no pre-activation gradient but G0 ever reaches HBM.
 * Outputs: de (with the residual gradient g + g2[dst]), G0 = dL/dh0 (row-major; its sender /
 * receiver segment sums are dP_s / dP_d, and dW_e = G0^T e goes to agn_wgrad), and per-block
 * partials (dW, db: agn_wgrad_reduce; LayerNorm: agn_colsum) summed in fixed order. de and G0
 * are bitwise those of the split path; dW / db / LayerNorm grads differ from it only in the fp32
 * order of the row sums. ---- */
typedef struct {
  int rows;                  /* edges (CSC order) */
  int nblk;                  /* grid size: agn_edge_bwd_blocks(rows) */
  const void* wpk[4];        /* packed A = W_l of W_e, Lin1, Lin2, Lin3 (agn_pack trans = 0, bf16) */
  const float* bias[4];      /* fp32 biases; bias[1..3] of Lin1..Lin3 (bias[0] unused: W_e has none) */
  const float* ln_g;         /* LayerNorm gamma [128] */
  const void* e;             /* [rows][128] the layer's edge input (CSC order) */
  const void* proj;          /* [N][256] P = [x W_s^T | x W_d^T + b] of the forward */
  const int32_t* src;        /* [rows] sender of each edge */
  const int32_t* dst;        /* [rows] receiver of each edge (row of proj's P_d half and of g2) */
  const void* g;             /* [rows][128] grad of e' or NULL (unused output) */
  const void* g2;            /* [N][128] dAgg (receiver-side grad) */
  void* de;                  /* [rows][128] out: dL/de incl. the residual */
  void* g0;                  /* [rows][128] out: dL/dh0 */
  float* dw_partial;         /* [3][nblk][128][128]: dW1..dW3 slabs (agn_wgrad slab order) */
  float* db_partial;         /* [3][nblk][128] */
  float* ln_partial;         /* [nblk][2][128]: sum g * xhat, sum g (LayerNorm weight / bias grads) */
  unsigned long long* stamps; /* diagnostics only (a -DAGN_EB_STAMPS build): NULL, or [2][8][8][16] */
  /* the forward's saves (agn_edge_forward32 with act[0] / stats): a1 = relu(h0) in AGN_TILED and
   * the LayerNorm (mean, rstd) [rows][2]. Given both, the kernel starts its recompute at Lin1 from
   * a1 (bitwise the values it would recompute) and reads no e, proj or src; NULL = recompute h0. */
  const void* a1;
  const float* stats;
  /* optional, read only without a1 / stats (with them a2 and a3 stay in registers and a1 is
   * re-read for its hand-off): [nblk][4][32][128] bf16 (32 KB per block,
   * agn_edge_bwd_scratch_bytes), the chain waves' a2 parked between the recompute and its hand-off
   * instead of recomputed a second time from a1 (a3 stays in registers either way). Outputs are
   * bitwise the same. Not the default: the slices do not stay in L2 and the launch is no faster
   * (DESIGN.md §9 round 6). */
  void* scratch;
  /* packed A = W_e^T (agn_pack trans = 1, bf16): de = G0 W_e + S reads it from L2 (round 6: W_e's
   * LDS image went to the hand-off ring) */
  const void* wtpk0;
  /* agn_encoder_bwd_fused only: the input's feature count (<= 16) and row stride (elements) */
  int xk;
  int xld;
} agn_edge_bwd_args;
int agn_edge_bwd_blocks(int rows);
size_t agn_edge_bwd_scratch_bytes(int nblk);
int agn_edge_bwd_fused(const agn_edge_bwd_args* a, void* stream);
/* The same fused backward for an encoder MLP (mlp.py:40-51 with 4 Linears, ReLU and LayerNorm on
 * k <= 16 input features: the node / edge encoders of bsms_mgn.py:138-139), when the input needs no
 * gradient: h0 = x W0^T + b0 is recomputed from the narrow input rows (e = x [rows or gathered
 * rows][xld], src = the gather index or NULL), S = g (g2 / dst / de / proj / wtpk0 unused), dW1..dW3,
 * db1..db3 and the LayerNorm partials as agn_edge_bwd_fused; G0 is written for dW0 = G0^T x and db0
 * (agn_wgrad). The forward then saves nothing (agn_mlp_forward without act / hpre / stats).
 * scratch as for agn_edge_bwd_fused (optional); grid agn_edge_bwd_blocks(rows). */
int agn_encoder_bwd_fused(const agn_edge_bwd_args* a, void* stream);
/* Device fault word of the persistent hand-off kernels (agn_edge_bwd_fused's LDS ring): the OR of
 * AGN_FAULT_* bits recorded since the last reset (0 = none). A set bit means a bounded wait gave
 * up and that launch's dW / db are wrong. Synchronises the device; reset != 0 clears the word. */
#define AGN_FAULT_RING_TIMEOUT 1
int agn_fault_status(int* value, int reset);
/* The same word without a device synchronisation: enqueues on `stream` a copy of the fault word
 * of agn_edge_bwd_fused into page-locked host memory (host_pinned[0]); the value is valid once
 * the stream reaches the copy. Nothing is reset. The production path enqueues one every
 * FAULT_POLL_EVERY (16) fused launches and reads it once its event has completed, and
 * GradAllReduce / the optimizer-step hook drain the last one (aerognn/core.py). */
int agn_fault_status_async(int* host_pinned, void* stream);
/* testing: sets the fault word (as a ring wait that gave up would), so the host-side polling can be
 * exercised without a real fault */
int agn_debug_set_fault(int value);
/* ---- arguments of the sum-trick edge chain's forward kernel (agn_edge_forward32) ---- */
typedef struct {
  int rows;                  /* edges (CSC order) */
  int nblk;                  /* grid size: agn_edge_fwd32_blocks(rows) */
  const void* wpk[4];        /* packed A = W_l of W_e, Lin1, Lin2, Lin3 (agn_pack trans = 0, bf16) */
  const float* bias[4];      /* fp32 biases; bias[1..3] of Lin1..Lin3 (bias[0] unused) */
  const float* ln_g;         /* LayerNorm gamma, beta [128] */
  const float* ln_b;
  const void* e;             /* [rows][128] edge input = the residual */
  const void* proj;          /* [N][256] P = [x W_s^T | x W_d^T + b] */
  const int32_t* src;
  const int32_t* dst;
  void* out;                 /* [rows][128] e' */
  void* act[3];              /* training saves: act[0] = a1 in AGN_TILED (rows padded to 32); act[1..2] NULL */
  void* hpre;                /* must be NULL */
  float* stats;              /* training saves: [rows][2] LayerNorm (mean, rstd), or NULL */
} agn_edge_fwd_args;
/* The chain on 32-edge tiles with 32x32x16 MFMAs, bitwise agn_mlp_forward's resident kernel
 * on the same operands: the forward of the training step (fused backward) and of inference.
 * Grid agn_edge_fwd32_blocks(rows). Replaces mlp.py:37-60 MLP.forward on EdgeBlockSum's chain
 * (mgnLayer.py:72-105, residual :205). With act[0] and stats set (training) it also saves the
 * first ReLU output a1 (AGN_TILED) and the LayerNorm statistics, which agn_edge_bwd_fused reads
 * instead of recomputing h0 from e and the projection rows. */
int agn_edge_fwd32_blocks(int rows);
int agn_edge_forward32(const agn_edge_fwd_args* a, void* stream);
/* dw[m][k] = sum_s dw_partial[s][m][k] (and db) for each desc: the fixed-order second stage
 * of agn_wgrad on caller-provided slabs (m, k <= 128 per desc here) */
int agn_wgrad_reduce(const agn_wgrad_batch* b, int nsplit, void* stream);

/* Node-row projections of the sum-trick edge block (mgnLayer.py:72-105, EdgeBlockSum's
 * src_lin / dst_lin applied per node instead of per edge), bf16, H = 128, persistent with the
 * packed weights resident in LDS (agn_pack layout, 64 KB):
 *   agn_proj_forward : out[r][0:256] = x[r] . [W_s; W_d]^T + bias   (wpk: 256 x 128 packed)
 *   agn_proj_backward: dx[r] += dps[r] . W_s + dpd[r] . W_d          (wtpk: 128 x 256 packed)
 * Bitwise identical to agn_mlp_forward with nlin = 1 on the same operands. Rows 16-B aligned. */
int agn_proj_forward(int rows, const void* x, int x_ld, const void* wpk, const float* bias, void* out, int out_ld,
                     void* stream);
int agn_proj_backward(int rows, const void* dps, const void* dpd, int dp_ld, const void* wtpk, void* dx, int dx_ld,
                      void* stream);

/* ---- device data preparation (dataset.py:39-106, :358-409; train.py:50-51) ----
 * agn_edge_features: out[i] = [pos[dst]-pos[src], |pos[dst]-pos[src]|] of edge e = perm ? perm[i] : i
 *   (i < ne output rows; edge_index int64 [2][e_total], perm int64), optionally normalised
 *   (v - mean) / std per column; [ne][pdim + 1] fp32.
 * agn_normalize: out = (x - mean) / std per column (inverse: x * std + mean, denormalize_predictions).
 * agn_col_stats: torch.std_mean(x, dim=0) (unbiased: NaN std for n = 1) of an [n][k] fp32 matrix, std clamped
 *   >= eps as torch.clamp does (a NaN stays NaN);
 *   deterministic fp64 two-pass; scratch = agn_col_stats_temp_bytes(n, k).
 * agn_collate: PyG Batch of B meshes concatenated row-wise: edge_index (in place) += the node offset
 *   of each edge's mesh, batch[v] = mesh of node v; edge_off / node_off exclusive prefix sums [B + 1]. */
int agn_edge_features(int ne, int64_t e_total, int pdim, const int64_t* edge_index, const float* pos, int pos_ld,
                      const int64_t* perm, const float* mean, const float* std, float* out, void* stream);
int agn_normalize(int n, int k, const float* x, int ld, const float* mean, const float* std, float* out, int out_ld,
                  int inverse, void* stream);
size_t agn_col_stats_temp_bytes(int n, int k);
int agn_col_stats(int n, int k, const float* x, int ld, float* mean, float* std, float eps, void* scratch,
                  void* stream);
int agn_collate(int B, int64_t ne, int64_t nn, const int64_t* edge_off, const int64_t* node_off, int64_t* edge_index,
                int64_t* batch, void* stream);

/* ---- float64 mode (train.py:20-40 precision "double" / "float64"): the MLP / GMP path in fp64
 * on plain LDS-tiled FMA kernels (csrc/f64.hip); graph ops take dtype AGN_F64. */
typedef struct {
  const double* a;      /* operand rows: row r is a + (aidx ? aidx[r] : r) * lda, k columns */
  const int32_t* aidx;  /* NULL, or gathered rows (x[src] / x[dst] of the concat edge MLP) */
  int lda, k;
  const double* w;      /* B(j, n) = transw ? w[n * ldw + j] : w[j * ldw + n] */
  int ldw, transw;
} agn_f64_seg;
typedef struct {
  int rows, n;          /* out [rows][n] */
  int nseg;             /* <= 3 */
  agn_f64_seg seg[3];
  const double* bias;   /* [n] or NULL */
  const double* add[2]; /* NULL or addends: add[q] + (add_idx[q] ? add_idx[q][r] : r) * add_ld[q] */
  const int32_t* add_idx[2];
  int add_ld[2];
  const double* mask;   /* NULL, or the activation backward: mask_act 0: out = 0 where mask <= 0
                           (ReLU on the saved activation); 1 + AGN_ACT_*: out *= f'(mask), mask = the
                           saved pre-activation */
  int mask_ld;
  int relu;             /* 0: none; 1: out = max(out, 0); 1 + AGN_ACT_*: out = f(out) */
  double* out;
  int out_ld;
  int mask_act;
  double* pre_out;      /* NULL, or the value before the activation (relu > 1) is also written here */
  int pre_ld;
  int _pad3;
} agn_f64_gemm_args;
/* out = f?(mask?(sum_seg A_seg B_seg + bias + add0 + add1)). Linear forward: transw = 1 (w = W
 * + column offset, ldw = in_features); input gradient: transw = 0. mlp.py:40-51, mgnLayer.py:97-103 */
int agn_f64_gemm(const agn_f64_gemm_args* a, void* stream);
typedef struct {
  int rows, m, k;
  const double* g; int ldg;                  /* [rows][m] */
  const double* x; int ldx;                  /* [rows][k], rows gathered by xidx if not NULL */
  const int32_t* xidx;
  double* dw; int ldw;                       /* [m][k] = g^T x (overwritten) */
  double* db;                                /* [m] = colsum g, or NULL */
} agn_f64_wgrad_args;
size_t agn_f64_wgrad_scratch_bytes(const agn_f64_wgrad_args* a);
int agn_f64_wgrad(const agn_f64_wgrad_args* a, void* scratch, void* stream);
/* torch.nn.LayerNorm over the last n <= 1024 features (biased variance), y = ... + resid */
int agn_f64_layernorm_fwd(int rows, int n, const double* x, int ldx, const double* gamma, const double* beta,
                          const double* resid, int ldr, double* y, int ldy, double* mean, double* rstd, double eps,
                          void* stream);
size_t agn_f64_layernorm_bwd_scratch_bytes(int rows, int n);
int agn_f64_layernorm_bwd(int rows, int n, const double* dy, int lddy, const double* x, int ldx, const double* mean,
                          const double* rstd, const double* gamma, double* dx, int lddx, double* dgamma,
                          double* dbeta, void* scratch, void* stream);

#ifdef __cplusplus
}
#endif
#endif
