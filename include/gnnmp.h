/*
 * gnnmp.h — C ABI of the MI355X (gfx950) GNN message-passing library `libgnnmp.so`.
 *
 * This is the drop-in boundary for the one hot path of elliptic-gnn-project:
 * the neighbour aggregation that `torch_geometric.nn.{SAGEConv,GCNConv,GATConv}`
 * perform inside `src/models/gnn.py` (imported at gnn.py:8, called at
 * gnn.py:28,31,49,52,72,75,187,193).  PyG 2.5.3 (the CI pin,
 * .github/workflows/ci.yml:17,39) is not vendored in the reference; every entry
 * point below names the PyG operation it replaces.
 *
 * Conventions
 *  - All buffers are device pointers owned by the caller.  The library never
 *    allocates or frees device memory; scratch comes from a caller-provided
 *    workspace whose size is queried first.
 *  - Feature matrices are row-major [rows, F] with a leading dimension `ld`
 *    (elements).  Outputs are fully overwritten (no zero-init contract).
 *  - Graph arrays are int32 (N, E < 2^31).  `edge_index` is PyG's [2, E] int64
 *    layout: row 0 = source j, row 1 = target i (flow source_to_target).
 *  - Every launch goes on the caller's stream; no entry point synchronises the
 *    host except gnn_graph_build's optional stats read (documented there).
 *  - Errors: a gnn_status is returned; gnn_last_error() gives a thread-local
 *    message.  Reductions are atomic-free: results are bitwise reproducible.
 */
#ifndef GNNMP_H_
#define GNNMP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNNMP_ABI_VERSION 26

typedef struct ihipStream_t* gnn_stream_t; /* == hipStream_t */

typedef enum {
  GNN_OK = 0,
  GNN_ERR_INVALID_ARG = 1,
  GNN_ERR_INDEX_OUT_OF_RANGE = 2, /* PyG: IndexError from index_select */
  GNN_ERR_HIP = 3,
  GNN_ERR_WORKSPACE = 4,
  GNN_ERR_UNSUPPORTED = 5
} gnn_status;

/* Self-loop handling applied while building a graph plan. */
typedef enum {
  GNN_LOOPS_KEEP = 0,    /* SAGEConv: edges used exactly as given (duplicates and loops kept) */
  GNN_LOOPS_REPLACE = 1  /* GCNConv add_remaining_self_loops / GATConv remove_self_loops +
                            add_self_loops: drop every existing loop, then one loop per node,
                            placed LAST in its CSR row and CSC column (PyG appends loops). */
} gnn_loop_mode;

/*
 * A graph plan: CSR by destination (aggregation, forward) and CSC by source
 * (transpose, backward), both stable in PyG edge order.
 */
/*
 * Long-segment split of one plan direction (see gnn_split_build).  Aggregations over a
 * split direction run the truncated segments in the main pass, reduce the remaining pieces
 * of long segments into a caller-provided partial buffer, and combine them in piece order.
 */
typedef struct {
  int32_t seg_len;            /* T: slots per piece */
  int32_t reserved;
  int64_t num_long;           /* segments with more than T slots */
  int64_t num_pieces;         /* pieces of the long segments (ceil(deg / T) each) */
  const int32_t* ptr;         /* [N+1] segment pointer, every segment truncated to <= T slots */
  const int32_t* nbr;         /* truncated segments' neighbours (PyG order kept) */
  const int32_t* piece0;      /* [N] partial-sum row of piece 0 of a long segment, -1 if short */
  const int32_t* piece_seg;   /* [num_pieces] segment of each piece */
  const int32_t* long_seg;    /* [num_long] the long segments */
  const int32_t* order;       /* optional [N]: ptr/nbr position i holds segment order[i] (degree
                                 order, longest first, stable); NULL: position i = segment i */
} gnn_split;

typedef struct {
  int64_t num_nodes;
  int64_t num_slots;        /* stored edges (after loop handling) */
  const int32_t* rowptr;    /* [N+1] CSR by target i */
  const int32_t* col;       /* [S]   source j of each CSR slot */
  const int32_t* colptr;    /* [N+1] CSC by source j */
  const int32_t* row;       /* [S]   target i of each CSC slot */
  const int32_t* csc2csr;   /* [S]   CSR slot holding the same edge as each CSC slot */
  const gnn_split* csr_split; /* optional (NULL): long-row split of the CSR direction */
  const gnn_split* csc_split; /* optional (NULL): long-column split of the CSC direction */
} gnn_graph;

int gnn_abi_version(void);
const char* gnn_status_string(gnn_status s);
const char* gnn_last_error(void);

/* ------------------------------------------------------------------------ */
/* K0  graph plan build  (replaces the implicit per-call index handling of
 *     MessagePassing.propagate, and remove/add_(remaining_)self_loops)      */
/* ------------------------------------------------------------------------ */
gnn_status gnn_graph_workspace_size(int64_t num_nodes, int64_t num_edges, size_t* bytes);

/*
 * Build a plan from edge_index [2,E] int64 (contiguous).  Output arrays must
 * hold S_max = E (KEEP) or E + N (REPLACE) slots; rowptr/colptr N+1.
 * csr_eid[s] = PyG edge id of CSR slot s (original id; loop of node i = E + i).
 * stats (device int32[4], zeroed by this call): {S, n_input_loops, n_bad_index, 0}.
 * A non-zero n_bad_index means some index was outside [0, N): the plan is invalid
 * (PyG raises IndexError); the caller reads stats after the stream completes.
 */
gnn_status gnn_graph_build(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                           gnn_loop_mode loops, int32_t* rowptr, int32_t* col, int32_t* csr_eid,
                           int32_t* colptr, int32_t* row, int32_t* csc2csr, int32_t* stats,
                           void* workspace, size_t workspace_bytes, gnn_stream_t stream);

/*
 * K0b  long-segment split of one direction (ptr/nbr = rowptr/col or colptr/row).
 * gnn_split_count writes {S_trunc, num_long, num_pieces} to device int64 counts[3] (the
 * caller reads them after the stream completes and sizes the outputs: tptr N+1, tnbr S_trunc,
 * piece0 N, piece_seg num_pieces, long_seg num_long).  gnn_split_build fills them; with
 * order (N entries, optional) the truncated tptr/tnbr are laid out in degree order (see
 * gnn_split.order) — the lane-group gather (8 < F <= 32·vec) runs its main pass in that order.
 */
gnn_status gnn_split_workspace_size(int64_t num_segs, size_t* bytes);
gnn_status gnn_split_count(const int32_t* ptr, int64_t num_segs, int32_t seg_len, int64_t* counts,
                           gnn_stream_t stream);
gnn_status gnn_split_build(const int32_t* ptr, const int32_t* nbr, int64_t num_segs, int32_t seg_len,
                           int32_t* tptr, int32_t* tnbr, int32_t* piece0, int32_t* piece_seg,
                           int32_t* long_seg, int32_t* order, void* workspace, size_t workspace_bytes,
                           gnn_stream_t stream);

/* deg[i] = number of CSR slots of i as float (PyG `count` / `deg`, gnn.py:49 via SAGEConv mean). */
gnn_status gnn_in_degree_f32(const gnn_graph* g, float* deg, gnn_stream_t stream);

/* K3  gcn_norm (PyG torch_geometric.nn.conv.gcn_conv.gcn_norm, improved=False, add_self_loops=True):
 *     dinv[i] = deg_i^-1/2 (inf -> 0) on a GNN_LOOPS_REPLACE plan.  Edge weight of (j -> i) is
 *     dinv[j]*dinv[i], formed inside the aggregation kernels.  Replaces GCNConv.forward's norm. */
gnn_status gnn_gcn_norm_f32(const gnn_graph* g, float* dinv, gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* K1/K2/K4  segmented aggregation over a plan (atomic-free)                */
/* ------------------------------------------------------------------------ */
typedef enum {
  GNN_AGG_SUM = 0,       /* y_r = sum_k x[nbr_k]                                          */
  GNN_AGG_MEAN = 1,      /* y_r = (sum_k x[nbr_k]) / max(nodew[r],1)  — SAGEConv aggr='mean' fwd (K1) */
  GNN_AGG_MEAN_BWD = 2,  /* y_r = sum_k x[nbr_k] / max(nodew[nbr_k],1) — mean backward over CSC (K2)  */
  GNN_AGG_GCN = 3,       /* y_r = sum_k (nodew[nbr_k]*nodew[r]) * x[nbr_k] — GCNConv propagate (K4)    */
  GNN_AGG_EDGE_W = 4     /* y_r = sum_k ew[slot_k, head(f)] * x[nbr_k, f] — GAT alpha-weighted (K5/K6) */
} gnn_agg_mode;

typedef struct {
  gnn_agg_mode mode;
  int32_t transpose;      /* 0: iterate CSR rows (targets gather sources); 1: CSC (sources gather targets) */
  const float* nodew;     /* per-node weights (deg for MEAN*, dinv for GCN) */
  const float* ew;        /* EDGE_W: per-CSR-slot weights [S, heads] */
  int32_t heads;          /* EDGE_W: feature f uses head f / (F / heads) */
  const float* addend;    /* optional [rows, F] added after the aggregation (ld_add) */
  int64_t ld_add;
  const float* bias;      /* optional [F] */
  int32_t relu;           /* apply max(.,0) last */
  float* part;            /* partial sums for a split direction: >= num_pieces * F floats; NULL or
                             too small -> the direction is aggregated unsplit */
  size_t part_bytes;
  float dropout_p;        /* > 0: F.dropout after bias / ReLU, element r*F + f kept by the counter
                             hash of gnn_gemm_nt_params (oracle/dropout_hash.py), kept values
                             scaled by 1/(1-p) — GCNNet's hidden layers (src/models/gnn.py:29-30) */
  uint64_t seed;
  const int64_t* seed_ptr; /* optional device counter: seed = *seed_ptr * 0x9E3779B97F4A7C15 + seed */
  const float* addend2;   /* optional (ABI 20, f32 only): a second [rows, F] term added after addend
                             (ld_add2) — a residual branch's gradient summed in the same store
                             (SAGE-ResBN's identity residual: dx = meanᵀ(dG_l) + dG_r + dr) */
  int64_t ld_add2;
} gnn_agg_params;

/* Generic fp32 aggregation: y[r, 0:F] for r in [0, N). */
gnn_status gnn_aggregate_f32(const gnn_graph* g, const gnn_agg_params* p, const float* x,
                             int64_t ldx, int64_t F, float* y, int64_t ldy, gnn_stream_t stream);

/* bf16-storage form: x and y hold bf16 ([rows, F], ld in elements), f32 accumulation in plan
 * order, y rounded once (RNE).  Modes SUM / MEAN / MEAN_BWD / GCN (no EDGE_W); addend f32. */
gnn_status gnn_aggregate_bf16(const gnn_graph* g, const gnn_agg_params* p, const void* x, int64_t ldx,
                              int64_t F, void* y, int64_t ldy, gnn_stream_t stream);

/* Split images ("planes"): an f32 matrix held as three bf16 planes hi / mid / lo with
 * v = hi + mid + lo exactly (hi = RNE(v), mid = RNE(v - hi), lo = RNE(v - hi - mid)); plane p
 * at img + p*plane_stride elements, element (r, c) at r*ld + c.  The split-bf16 GEMMs read them
 * instead of splitting f32 operands in-kernel (gnn_gemm_nt_params / gnn_gemm_tn_params .a_planes).
 *
 * gnn_split_planes_f32: columns [col0, col0 + width) of rows [0, rows) <- planes of x [rows, F]
 * (zeros at columns >= F; width, col0, ld, plane_stride even). */
gnn_status gnn_split_planes_f32(const float* x, int64_t ldx, int64_t rows, int64_t F, void* img, int64_t ld,
                                int64_t plane_stride, int64_t col0, int64_t width, gnn_stream_t stream);
/* K1 with a split-image store: columns [0, width) of img <- planes of mean_{j->i} x[j]
 * (SAGEConv aggr='mean', the same arithmetic as gnn_sage_mean_fwd_f32), zeros at columns >= F.
 * Wide rows only (even F, 32 < F / vec with vec = 4 or 2, width / vec <= 128): UNSUPPORTED otherwise. */
gnn_status gnn_sage_mean_fwd_planes(const gnn_graph* g, const float* deg, const float* x, int64_t ldx, int64_t F,
                                    void* img, int64_t ld, int64_t plane_stride, int64_t width,
                                    gnn_stream_t stream);

/* Half-pair images: an f32 matrix held as TWO f16 planes of its PRE-SCALED values
 * u = v * 2^scale_exp:  hi = RNE_f16(u), lo = RNE_f16((u - hi) * 2^11), so u = hi + 2^-11 lo to
 * 2^-22 |u| while hi and (u - hi) * 2^11 are f16 normals, i.e. |u| >= 2^-13 (below that the pair
 * holds u to an absolute 2^-36).  The caller picks scale_exp per matrix so that its largest
 * magnitude lands in [2^13, 2^14): scale_exp = 14 - E with max|v| in [2^(E-1), 2^E) (0 for an
 * all-zero matrix; |scale_exp| <= 100).  Every value within 2^-26 of the matrix's largest then
 * keeps the full 2^-22 relative precision, whatever the matrix's overall magnitude (ABI 19: the
 * unscaled images of ABI 18 lost it below |v| ~ 2^-13).  |u| must stay below 2^15 (f16 range with
 * headroom for the agg half, a mean of the x rows).  The consuming GEMMs undo the scale exactly
 * (gnn_gemm_nt_params / gnn_gemm_tn_params .planes_exp, a power of two in their epilogues).  The
 * half-pair GEMMs (planes_format = GNN_PLANES_HALF_PAIR) run 3 f16 products per product instead
 * of the split-bf16 form's 6 and move 4 B per element instead of 6.  Otherwise the same layout and
 * arguments as the split-bf16 functions above. */
gnn_status gnn_split_h2_f32(const float* x, int64_t ldx, int64_t rows, int64_t F, void* img, int64_t ld,
                            int64_t plane_stride, int64_t col0, int64_t width, int32_t scale_exp,
                            gnn_stream_t stream);
/* gnn_sage_mean_fwd_h2: K1 with a half-pair store of mean_{j->i} x[j] * 2^scale_exp (the mean
 * rounded as gnn_sage_mean_fwd_f32 rounds it, then scaled exactly; scale_exp = the exponent of
 * the image's x half, so |agg * 2^scale_exp| <= max|x * 2^scale_exp|).  It optionally also writes
 * the dropout keep bits of the NT that consumes the
 * image (keep_mask != NULL, [num_nodes][4] uint32, 16-byte aligned; the NT reads the words of
 * ceil(num_nodes / 32) * 32 rows, clamping the row index into [0, num_nodes)): bit c of
 * keep_mask[r*4 + c/32] = keep_elem(seed', r*mask_cols + c) with seed' the NT's (seed, seed_ptr)
 * rule — the mask the NT would hash itself, computed where the gather leaves the VALU idle
 * (gnn_gemm_nt_params.keep_mask).
 * prep_b (optional): the params of the half-pair NT that reads this image (a_planes == img and
 * planes_exp == scale_exp); its B-image prep (gnn_gemm_nt_prep_b) runs inside this launch, on
 * extra blocks beside the gather, for a later gnn_gemm_nt_f32 of the same params with
 * b_ready = 1.  UNSUPPORTED when the params do not select the half-pair NT.
 * hub (optional, ABI 21; NULL or num_long == 0: one wave per 16 rows throughout): the rows r with
 * deg[r] > hub->seg_len (hub->long_seg, num_long of them) are each walked by a block of their own
 * (4 waves over interleaved 8-slot groups, summed in wave order) instead of by the wave holding
 * them; hub->ptr / nbr are the CSR with those rows' slots removed (natural order: order and
 * piece0 NULL; num_pieces, piece_seg unused).  For small graphs (a strong-scaling shard), where
 * the one wave walking a hub row is the launch's tail.  Changes the hub rows' summation order
 * (within the mean's rounding), not the other rows'.  hub->piece_seg (optional): [num_pieces + 1]
 * non-decreasing row boundaries from 0 to num_nodes, wave k of the main pass taking rows
 * [piece_seg[k], piece_seg[k + 1]) (at most 64; balanced by slots instead of 16 rows each). */
struct gnn_gemm_nt_params;
gnn_status gnn_sage_mean_fwd_h2(const gnn_graph* g, const float* deg, const float* x, int64_t ldx, int64_t F,
                                void* img, int64_t ld, int64_t plane_stride, int64_t width, int32_t scale_exp,
                                uint32_t* keep_mask, int64_t mask_cols, float dropout_p, uint64_t seed,
                                const uint64_t* seed_ptr, const struct gnn_gemm_nt_params* prep_b,
                                const gnn_split* hub, gnn_stream_t stream);
typedef enum {
  GNN_PLANES_SPLIT_BF16 = 0,  /* 3 bf16 planes hi / mid / lo (gnn_split_planes_f32) */
  GNN_PLANES_HALF_PAIR = 1    /* 2 f16 planes hi / lo (gnn_split_h2_f32) */
} gnn_planes_format;

/* The SAGE output layer's mean and the training loss in ONE pass (ABI 19): logits = mean_{j->i}
 * z[j, 0:C] + z[i, C:2C] + bias (SAGEConv transform-first: z = h·[W_l ; W_r]ᵀ, gnn.py:49-53) —
 * gnn_aggregate_f32(MEAN, addend, bias)'s arithmetic — and, in the same kernel's epilogue, the
 * masked class-weighted cross entropy of those logits (gnn_masked_ce_f32: dlogits, per-256-row loss
 * partials in `workspace`, `loss` = Σ partials · inv_denom or left to gnn_masked_ce_finish /
 * gnn_adam_group.loss_partial when NULL), bit for bit as the two calls produce them.  Replaces
 * the F = 2 aggregation + the CE launch of the training step (src/train_gnn.py:192-199).
 * 1 <= C <= 4, ldz >= 2C; workspace: gnn_masked_ce_workspace_size(num_nodes).  u (optional, ABI 20,
 * [N, C], ldu >= C): dlogits / max(deg, 1) per row — the transposed mean's per-slot term, so the
 * backward's meanᵀ(dlogits) is a plain CSC sum of u (gnn_aggregate_f32 SUM, transpose), bit for bit
 * the MEAN_BWD result, without the per-slot degree gather and division.  colsum (optional, ABI 21):
 * dlogits' per-256-row-block column sums as gnn_masked_ce_colsum_f32 writes them (the output
 * bias gradient through gnn_colsum_finish_f32: SAGE-ResBN's output conv). */
gnn_status gnn_sage_out_mean_ce_f32(const gnn_graph* g, const float* deg, const float* z, int64_t ldz, int32_t C,
                                    const float* bias, float* logits, int64_t ldo, const int64_t* y,
                                    const uint8_t* mask, const float* class_w, float inv_denom, float* dlogits,
                                    int64_t ld_d, float* u, int64_t ldu, float* colsum, float* loss, void* workspace,
                                    size_t workspace_bytes, gnn_stream_t stream);

/* Named forms of the above (what an FFI binding of SAGEConv would call). */
gnn_status gnn_sage_mean_fwd_f32(const gnn_graph* g, const float* deg, const float* x, int64_t ldx,
                                 int64_t F, float* out, int64_t ldo, gnn_stream_t stream);
gnn_status gnn_sage_mean_bwd_f32(const gnn_graph* g, const float* deg, const float* dout,
                                 int64_t ld_dout, int64_t F, float* dx, int64_t ld_dx,
                                 gnn_stream_t stream);

/* Explain mode (PyG MessagePassing.propagate with `explain` on: every message multiplied by
 * edge_mask[e] before aggregation; driven by GNNExplainer, src/analysis/explain.py:593-672).
 * Forward and x-gradient run as GNN_AGG_EDGE_W with the mask as slot weight; this entry point
 * gives the mask gradient: out[eid ? eid[s] : s] = <a[r], b[col[s]]> / max(nodew[r], 1)
 * (nodew NULL: / 1) for every CSR slot s of row r — for SAGEConv's mean a = dOut, b = x. */
gnn_status gnn_edge_dot_f32(const gnn_graph* g, const int32_t* eid, const float* nodew, const float* a,
                            int64_t lda, const float* b, int64_t ldb, int64_t F, float* out,
                            gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* K5/K6  GATConv edge softmax + aggregation (PyG GATConv.edge_update/message, utils.softmax) */
/* ------------------------------------------------------------------------ */
/* a_src[n,h] = <xh[n,h,:], att_src[h,:]>, a_dst likewise. xh is [N, H*C] (ld_xh). */
gnn_status gnn_gat_scores_f32(int64_t N, int32_t H, int32_t C, const float* xh, int64_t ld_xh,
                              const float* att_src, const float* att_dst, float* a_src,
                              float* a_dst, gnn_stream_t stream);

/* Fused forward over a GNN_LOOPS_REPLACE plan: e = leaky_relu(a_src[j]+a_dst[i], slope);
 * alpha = exp(e - max_i) / (sum_i exp + 1e-16); out[i] = sum alpha * xh[j]
 * (concat: [N,H*C]; else head-mean [N,C]) + bias.  alpha saved per CSR slot [S,H]. */
gnn_status gnn_gat_fwd_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                           const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                           const float* bias, float* alpha, float* out, int64_t ldo,
                           gnn_stream_t stream);

/* Fused forward, scores in-kernel: a_src / a_dst are formed from the gathered xh rows and the
 * attention vectors (no gnn_gat_scores_f32 pass; both are written out for the backward), and
 * GATNet's hidden-layer activation is applied on the store (src/models/gnn.py:72-74):
 *   out = dropout(act(sum_j alpha_ij xh[j] + bias))   act = GNN_ACT_NONE | GNN_ACT_ELU (alpha 1)
 * dropout as in gnn_gemm_nt_params: keep iff hash(seed, row*F_out + col) < 1-p, kept / (1-p).
 * Same softmax as gnn_gat_fwd_f32 (one-pass online max / sum, merged in a fixed order). */
typedef enum { GNN_ACT_NONE = 0, GNN_ACT_ELU = 1 } gnn_act;
typedef struct {
  int32_t heads, chans, concat;
  float slope;
  const float* xh; int64_t ld_xh;         /* [N, H*C] */
  const float* att_src; const float* att_dst;  /* [H*C] */
  const float* bias;                      /* optional [F_out] */
  gnn_act act;
  float dropout_p;                        /* 0 = off */
  uint64_t seed; const uint64_t* seed_ptr; /* as gnn_gemm_nt_params */
  float* a_src; float* a_dst;             /* out [N, H] */
  float* alpha;                           /* out [S, H] */
  float* out; int64_t ldo;                /* out [N, F_out] */
  const float* edge_w;                    /* optional [S]: explain mode (PyG propagate with
                                             `_explain`): every message alpha * xh[j] of CSR slot s is
                                             multiplied by edge_w[s] after the softmax */
  const float* proj; int32_t nproj;       /* optional (ABI 24, concat layers): z = out · projᵀ written */
  float* z; int64_t ldz;                  /* beside the store, proj [nproj, H·C] (16-byte aligned,
                                             nproj <= 4) — GATNet's output conv's lin (gnn.py:75) on the
                                             hidden layer's stored rows, so its input is never read back */
} gnn_gat_fwd_params;
gnn_status gnn_gat_fwd_fused_f32(const gnn_graph* g, const gnn_gat_fwd_params* p, gnn_stream_t stream);
/* GATNet's output conv (src/models/gnn.py:67,75: heads 1, C <= 2, concat False, no act / dropout /
 * edge_w) in the narrow slot-parallel form, optionally with the masked CE in the same launch
 * (round 6, ABI 22): out, a_src, a_dst and alpha exactly as gnn_gat_fwd_fused_f32 defines them
 * (online softmax per row; fp32-close, not bitwise, to the lane-group kernel), then — y non-NULL —
 * gnn_masked_ce_f32 of the logits with its workspace contract (loss NULL: partials deferred),
 * dlogits, and colsum (optional) the per-256-row-block column sums of dlogits as
 * gnn_masked_ce_colsum_f32 writes them.  N >= 1. */
gnn_status gnn_gat_out_ce_f32(const gnn_graph* g, const gnn_gat_fwd_params* p, const int64_t* y, const uint8_t* mask,
                              const float* class_w, float inv_denom, float* dlogits, int64_t ld_d, float* colsum,
                              float* loss, void* workspace, size_t workspace_bytes, gnn_stream_t stream);

/* Gradient through y = dropout(act(pre)) from y itself (F.elu / F.dropout backward, gnn.py:73-74):
 * dpre = dy * keep * 1/(1-p) * act'(pre), ELU' = 1 for y > 0 else exp(pre) = y*(1-p) + 1.
 * [N, F]; dpre may alias dy. */
gnn_status gnn_gat_act_bwd_f32(int64_t N, int64_t F, gnn_act act, float dropout_p, uint64_t seed,
                               const uint64_t* seed_ptr, const float* y, int64_t ldy, const float* dy,
                               int64_t lddy, float* dpre, int64_t ld_dpre, gnn_stream_t stream);

/* Backward.  dout is [N,H*C] (concat) or [N,C].  Produces dxh [N,H*C] (includes the score
 * paths through att_src/att_dst), d_att_src/d_att_dst [H*C].  workspace from
 * gnn_gat_bwd_workspace_size. */
gnn_status gnn_gat_bwd_workspace_size(int64_t N, int64_t S, int32_t H, int32_t C, size_t* bytes);
gnn_status gnn_gat_bwd_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                           const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                           const float* att_src, const float* att_dst, const float* alpha,
                           const float* dout, int64_t ld_dout, float* dxh, int64_t ld_dxh,
                           float* d_att_src, float* d_att_dst, void* workspace,
                           size_t workspace_bytes, gnn_stream_t stream);

/* Backward of a hidden GATConv whose output went through dropout(act(.)) in the forward store
 * (gnn_gat_fwd_fused_f32 with act / dropout_p; concat heads): dy is the gradient of the stored
 * y; d pre = dy * keep / (1-p) * act'(pre) (gnn_gat_act_bwd_f32's formula) is formed inside the
 * rows pass as each row is loaded and written to dpre [N, H*C] (the cols pass and the bias
 * gradient read it); otherwise as gnn_gat_bwd_f32.  Replaces the act / dropout backward of
 * GATNet's hidden layers (src/models/gnn.py:73-74) fused with GATConv's. */
gnn_status gnn_gat_bwd_act_f32(const gnn_graph* g, int32_t H, int32_t C, float slope, const float* xh,
                               int64_t ld_xh, const float* a_src, const float* a_dst, const float* att_src,
                               const float* att_dst, const float* alpha, gnn_act act, float dropout_p,
                               uint64_t seed, const uint64_t* seed_ptr, const float* y, int64_t ld_y,
                               const float* dy, int64_t ld_dy, float* dpre, int64_t ld_dpre, float* dxh,
                               int64_t ld_dxh, float* d_att_src, float* d_att_dst, void* workspace,
                               size_t workspace_bytes, gnn_stream_t stream);

/* (ABI 24) gnn_gat_bwd_act_f32 with dy given as dz · proj (dz [N, nproj], ld_dz; proj [nproj, H·C],
 * 16-byte aligned, nproj <= 4): the backward of a hidden layer whose output fed a projection
 * (gnn_gat_fwd_params.proj) — dy is formed as each row slice loads, never stored.
 * (ABI 25) dxh_rowmax (optional, [ceil(N / GNN_ROWMAX_ROWS)] uint32): also the float bits of max |dxh|
 * over each group of GNN_ROWMAX_ROWS rows — the g_rowmax of the weight-gradient TN of the layer's
 * lin (dW = dxhᵀ · x), which then skips its own pass over dxh. */
gnn_status gnn_gat_bwd_act_proj_f32(const gnn_graph* g, int32_t H, int32_t C, float slope, const float* xh,
                                    int64_t ld_xh, const float* a_src, const float* a_dst, const float* att_src,
                                    const float* att_dst, const float* alpha, gnn_act act, float dropout_p,
                                    uint64_t seed, const uint64_t* seed_ptr, const float* y, int64_t ld_y,
                                    const float* dz, int64_t ld_dz, const float* proj, int32_t nproj, float* dpre,
                                    int64_t ld_dpre, float* dxh, int64_t ld_dxh, float* d_att_src, float* d_att_dst,
                                    uint32_t* dxh_rowmax, void* workspace, size_t workspace_bytes,
                                    gnn_stream_t stream);

/* Explain-mode backward (messages scaled by edge_w[s], see gnn_gat_fwd_params.edge_w): as
 * gnn_gat_bwd_f32, plus d_edge_w[s] = sum_h alpha[s,h] * <dout_i(h), xh[j,h,:]> for every CSR slot. */
gnn_status gnn_gat_bwd_ew_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                              const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                              const float* att_src, const float* att_dst, const float* alpha,
                              const float* dout, int64_t ld_dout, float* dxh, int64_t ld_dxh,
                              float* d_att_src, float* d_att_dst, const float* edge_w, float* d_edge_w,
                              void* workspace, size_t workspace_bytes, gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* K7  fp32 MFMA GEMMs with the surrounding elementwise work fused in.      */
/*     Replace PyG Linear lin_l/lin_r/lin (gnn.py:20-23,41-44,64-67) and the  */
/*     F.relu + F.dropout between layers (gnn.py:29-30,50-51,73-74).          */
/* ------------------------------------------------------------------------ */
/* Element type of a feature buffer. */
typedef enum { GNN_DTYPE_F32 = 0, GNN_DTYPE_BF16 = 1 } gnn_dtype;

/* Arithmetic of the K7 GEMMs.  Both are fp32-accurate (inputs, outputs and accumulation f32). */
typedef enum {
  GNN_MATH_SPLIT_BF16 = 0, /* default: every f32 operand split into hi+mid+lo bf16 terms, 6 products on
                              v_mfma_f32_32x32x16_bf16 (dropped terms <= ~2^-23 relative per product);
                              used for the w1/w2 NT form and the TN kernel, else falls back to: */
  GNN_MATH_F32 = 1,        /* exact f32 MFMA (v_mfma_f32_32x32x2_f32, a k-ordered fmaf chain) */
  GNN_MATH_HALF_PAIR = 2   /* (ABI 23) f32 operands split in the kernel into half-pair f16 terms
                              (hi = RNE_f16(v·s), lo = RNE_f16((v·s − hi)·2^11)), 3 products on
                              v_mfma_f32_32x32x16_f16, 2^-22 relative per operand, with power-of-two
                              scales that keep every operand in f16 range: the NT per A row
                              (max_k |A[r,k]| < 2^E_r, A[r,:]·2^(14−E_r)) and per B column; the TN per
                              row block for A (from the NT's row_exp) and for G (a max|g| pass over
                              the block's rows).  Taken by the w1/w2 NT (N <= 128, k1, k2 multiples of
                              16, k1 + k2 <= 128, f32 A / C) and by the plain g-form TN given row_exp
                              (Nr % 4 == 0, 16-byte aligned g rows); any other call runs as
                              GNN_MATH_SPLIT_BF16 */
} gnn_gemm_math;
/* Skinny shapes run full-f32 VALU kernels whatever `math` says (the 2-class output layers,
 * gnn.py:23,66,124): NT with N <= 8 (K <= 384) or with K <= 8 (one A segment), f32 A/C and no
 * projection; TN with Nr <= 8 in the plain g form (no dz/proj, h or gout) and f32 A. */

typedef struct gnn_gemm_nt_params {
  int64_t M, N;                          /* C is [M, N] */
  const float* a1; int64_t lda1; int64_t k1;
  const float* a2; int64_t lda2; int64_t k2;   /* optional 2nd K segment: A = [A1 | A2] (k2 = 0: none) */
  const float* bt; int64_t ldb;          /* [k1+k2, N] row-major (Linear weight transposed), or NULL and: */
  const float* w1; const float* w2;      /* ... B read in place from PyTorch Linear weights W1 [N, k1], */
  int64_t ldw1, ldw2;                    /*     W2 [N, k2] (N <= 128): out = [A1|A2]·[W1|W2]ᵀ, no copy */
  float* c; int64_t ldc;                 /* output (may be NULL when only z is wanted) */
  const float* bias;                     /* [N] or NULL */
  int32_t relu;                          /* max(., 0) after bias */
  float dropout_p;                       /* after ReLU; 0 = off.  keep if hash(seed, row*N+col) < 1-p */
  uint64_t seed;                         /* per-call salt (the seed itself when seed_ptr is NULL) */
  const uint64_t* seed_ptr;              /* optional device counter: seed = *seed_ptr * golden + seed
                                            (graph-replay safe: bump the counter inside the graph) */
  const float* proj; int32_t nproj;      /* optional Z = C · projᵀ, proj [nproj, N], nproj <= 4, N <= 128 */
  float* z; int64_t ldz;
  int32_t math;                          /* gnn_gemm_math */
  void* workspace; size_t workspace_bytes; /* optional: the split-bf16 w1/w2 form pre-splits B here
                                            (gnn_gemm_nt_workspace_size) */
  int32_t a_dtype;                       /* gnn_dtype of A1/A2 (BF16: w1/w2 form; B rounded to bf16,
                                            one bf16 product, f32 accumulate — the bf16-storage path) */
  int32_t c_dtype;                       /* gnn_dtype of C (BF16 needs a_dtype BF16); z stays f32 */
  const float* mask;                     /* optional [M, N] (ldmask): C *= (mask > 0 ? mask_scale : 0)
                                            after the other epilogue steps — the ReLU + dropout
                                            backward of a saved activation (K <= 8 or N <= 8 shapes) */
  int64_t ldmask;
  float mask_scale;
  const void* a_planes;                  /* optional split image of [A1 | A2] (see gnn_split_planes_f32):
                                            A1 in columns [0, k1), A2 in [planes_col2, planes_col2 + k2),
                                            zeros elsewhere.  When the shape is one the split-image kernel
                                            takes (gnn_gemm_nt_planes_ok) A is read from it and a1 / a2 may
                                            be NULL; otherwise a1 / a2 are used (UNSUPPORTED if NULL). */
  int64_t planes_ld, planes_stride, planes_col2;
  int32_t planes_format;                 /* gnn_planes_format of a_planes (HALF_PAIR: 336-wide rows,
                                            1 <= N <= 128, N % 4 == 0; B per output column scaled by
                                            a power of two into f16 range, 3 f16 products) */
  const uint32_t* keep_mask;             /* optional (HALF_PAIR with dropout): the keep bits written by
                                            gnn_sage_mean_fwd_h2 for this call's seed / p / N; used
                                            instead of hashing every element in the epilogue */
  int32_t b_ready;                       /* image-A forms only: nonzero = workspace already holds the B
                                            image gnn_gemm_nt_prep_b wrote for these weights and shapes
                                            (the call launches only the GEMM) */
  int32_t planes_exp;                    /* HALF_PAIR (ABI 19): the image holds A * 2^planes_exp
                                            (gnn_split_h2_f32 scale_exp); C is unscaled exactly */
  float* colsum_part; int64_t colsum_cap; /* optional (ABI 21): the skinny-K form (k1 <= 8, k2 = 0,
                                            8 < N <= 256; UNSUPPORTED otherwise) also writes the column
                                            sums of the C it stores (after the whole epilogue), one row per
                                            block: colsum_part[b * N + n], b < gnn_gemm_nt_colsum_blocks;
                                            capacity colsum_cap floats.  gnn_colsum_finish_f32 then
                                            gives Σ_rows C — a layer's bias gradient without a pass over C */
  int32_t* row_exp;                      /* optional (ABI 23, GNN_MATH_HALF_PAIR form only): [M] per-row
                                            exponents E_r with max_k |[A1|A2][r,k]| < 2^E_r (0 for a zero
                                            row, 128 for a non-finite one) — the TN's A bound
                                            (gnn_gemm_tn_params.row_exp) for the same operand */
} gnn_gemm_nt_params;

/* C = epilogue([A1|A2] · Bt). */
gnn_status gnn_gemm_nt_colsum_blocks(const gnn_gemm_nt_params* p, int32_t* nb);  /* 0: no column sums */
gnn_status gnn_gemm_nt_workspace_size(int64_t N, int64_t k1, int64_t k2, size_t* bytes);
gnn_status gnn_gemm_nt_f32(const gnn_gemm_nt_params* p, gnn_stream_t stream);
/* The image-A forms' weight prep alone: writes the B image (split / half-pair / bf16 planes of
 * [w1 | w2]ᵀ, with the half-pair column scales) into p->workspace, for a later gnn_gemm_nt_f32 of
 * the same params with b_ready = 1.  Lets a caller run the prep on a second stream beside the
 * producer of A (it reads only the weights).  UNSUPPORTED (nothing launched) when the params do
 * not select an image-A kernel (gnn_gemm_nt_planes_ok). */
gnn_status gnn_gemm_nt_prep_b(const gnn_gemm_nt_params* p, gnn_stream_t stream);

typedef struct {
  int64_t M, Nr;                         /* dW is [Nr, k1+k2], Nr <= 128, k1+k2 <= 384 */
  const float* g; int64_t ldg;           /* G [M, Nr] ... */
  const float* dz; int64_t lddz;         /* ... or G = dz · proj (dz [M, nproj], proj [nproj, Nr]) */
  const float* proj; int32_t nproj;
  const float* h; int64_t ldh; float hscale;   /* optional: G *= (h > 0 ? hscale : 0) — ReLU+dropout bwd */
  float* gout; int64_t ldgout;           /* optional: store G */
  const float* a1; int64_t lda1; int64_t k1;
  const float* a2; int64_t lda2; int64_t k2;
  int32_t math;                          /* gnn_gemm_math */
  int32_t a_dtype;                       /* gnn_dtype of A1/A2 (BF16: G rounded to bf16, one product;
                                            needs M >= 16) */
  int32_t h_dtype;                       /* gnn_dtype of h */
  const void* a_planes;                  /* optional split image of [A1 | A2], as gnn_gemm_nt_params */
  int64_t planes_ld, planes_stride, planes_col2;
  int32_t planes_format;                 /* gnn_planes_format (HALF_PAIR: the dz form with h, 336-wide
                                            rows, or the plain g form over 336- / 176-wide rows; G scaled
                                            per row block by a power of two, 3 products) */
  int32_t g_dtype;                       /* gnn_dtype of g and gout (BF16: the bf16-image TN only; gout
                                            then holds the bf16-rounded G its MFMAs use) */
  int32_t planes_exp;                    /* HALF_PAIR (ABI 19): the image holds A * 2^planes_exp; dW is
                                            unscaled exactly */
  float* sq_partial;                     /* optional (ABI 20): the clip + Adam norm partials of `out`, for a
                                            call whose out holds every gradient of an optimizer group —
                                            per block b < nb of the ordered reduce (nb =
                                            gnn_gemm_tn_sq_blocks), over the out[j] with j outside
                                            [sq_skip_lo, sq_skip_hi): sq_partial[b] = Σ out[j]², sq_partial[nb + b]
                                            = the count of non-finite out[j]; sq_partial[2 nb] = *sq_step (the
                                            step count before the update).  Capacity sq_cap floats >= 2 nb + 1;
                                            hand them to gnn_clip_adam_f32 (gnn_adam_group.grad_sq_partial) */
  const float* sq_step;
  int64_t sq_skip_lo, sq_skip_hi, sq_cap;
  const int32_t* row_exp;                /* optional (ABI 23): [M] exponents bounding the rows of [A1|A2]
                                            (max_k |A[r,k]| < 2^row_exp[r]), as a GNN_MATH_HALF_PAIR NT of
                                            the same operand writes them; with math GNN_MATH_HALF_PAIR and
                                            the plain g form the TN runs in half-pair arithmetic */
  const uint32_t* g_rowmax;              /* optional (ABI 25), the plain g form over a half-pair image:
                                            [ceil(M / GNN_ROWMAX_ROWS)] float bits of max |G| over each
                                            group of GNN_ROWMAX_ROWS rows and all Nr columns (an upper
                                            bound is enough), as gnn_gat_bwd_act_proj_f32 writes them for
                                            its dxh: the TN takes its per-row-block power-of-two scale
                                            from these instead of a pass over its G rows.  Exact maxima
                                            give the scan's scale, so the result is bit-identical. */
  const gnn_graph* dz_graph;             /* optional (ABI 26), the half-pair dz form without gout: the TN
                                            itself forms dz[:, 0:dz_cols] = Σ over each row's CSC slots of
                                            dz_u[source, 0:dz_cols] — gnn_aggregate_f32(SUM, transpose) of
                                            dz_u, bit for bit — and writes it into dz before using it, so
                                            the caller skips that launch (the SAGE output layer's meanᵀ of
                                            u = dlogits / deg, gnn_sage_out_mean_ce_f32).  Inside its
                                            kernel when a row block is at most ~450 rows (a strong-scaling
                                            shard), else by that aggregation launched first.  1 <= dz_cols
                                            <= min(2, nproj), dz_graph->num_nodes == M; UNSUPPORTED outside
                                            that kernel.  gnn_gemm_tn_planes_ok returns 1 for such
                                            params only when the kernel forms the columns itself */
  const float* dz_u; int64_t ldu;
  int32_t dz_cols;
} gnn_gemm_tn_params;

/* Row-group granularity of gnn_gemm_tn_params.g_rowmax (ABI 25). */
#define GNN_ROWMAX_ROWS 16

/* Weight gradient dW = Gᵀ·[A1|A2] summed over all M rows (split-M slabs + ordered reduce).
 * out (contiguous): dW1 = Gᵀ·A1 [Nr, k1] | dW2 = Gᵀ·A2 [Nr, k2] | db = Σ_m G [Nr] |
 * (dz form) dWp = dzᵀ·h [nproj, Nr] | dzsum = Σ_m dz [nproj]. */
gnn_status gnn_gemm_tn_workspace_size(int64_t M, int64_t Nr, int64_t Kc, int32_t nproj, size_t* bytes);
gnn_status gnn_gemm_tn_f32(const gnn_gemm_tn_params* p, float* out, void* workspace, size_t workspace_bytes,
                           gnn_stream_t stream);
/* The number nb of norm partials a call with sq_partial writes for an out of n_out floats (ABI 20). */
gnn_status gnn_gemm_tn_sq_blocks(int64_t n_out, int32_t* nb);
/* 1 when the call would read A from p->a_planes (the f32 A operands are then not needed), else 0.
 * Split-image NT shapes (f32 C, the w1/w2 B form, N % 4 == 0, M >= 32; a ReLU, dropout or
 * projection epilogue needs relu + bias):
 *   image rows of 336 (the SAGE layer-1 [agg | x], 166 + 166 padded to 168 each), 64 < N <= 128;
 *   image rows of 176 (one input of <= 176 columns: the GCN / GAT layer-1 x), 1 <= N <= 128;
 *   a half-pair image (planes_format HALF_PAIR) of 336-wide rows, 1 <= N <= 128.
 * TN image rows of 32..336 (multiple of 16), f32 h; half-pair: the dz form with h, 336-wide rows,
 * or (ABI 19) the plain g form — g given, no dz / h / gout, 16-byte aligned g rows — over 336- or
 * 176-wide rows (gnn_gemm_tn_planes_ok).  Both need the planes to span < 2 GiB
 * and C / z below 2 GiB. */
int gnn_gemm_nt_planes_ok(const gnn_gemm_nt_params* p);
int gnn_gemm_tn_planes_ok(const gnn_gemm_tn_params* p);

/* ------------------------------------------------------------------------ */
/* Dense helpers used by the fused conv paths                               */
/* ------------------------------------------------------------------------ */
/* out[c] = sum_r x[r, c]  (bias gradients; deterministic two-stage column sum). */
gnn_status gnn_colsum_workspace_size(int64_t rows, int64_t F, size_t* bytes);
/* out[f] = Σ_b part[b * F + f] over b < nblk in gnn_colsum_f32's fixed order (ABI 21: the column
 * sums a skinny-K gnn_gemm_nt_f32 call wrote, gnn_gemm_nt_params.colsum_part) */
gnn_status gnn_colsum_finish_f32(const float* part, int32_t nblk, int64_t F, float* out, gnn_stream_t stream);
gnn_status gnn_colsum_f32(int64_t rows, int64_t F, const float* x, int64_t ldx, float* out,
                          void* workspace, size_t workspace_bytes, gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* K12 SAGEResBNNet layer tail, training mode (src/models/gnn.py:182-194):   */
/*     h = dropout(relu(BatchNorm1d(z))) + r,   r = res_proj(h_prev)          */
/* Replaces nn.BatchNorm1d.forward (batch statistics + running-stat update),  */
/* F.relu, F.dropout and the residual add, and their backward passes.         */
/* ------------------------------------------------------------------------ */
/* Workspace of gnn_bn_stats_f32 / gnn_bn_act_bwd_reduce_f32 for C channels. */
gnn_status gnn_bn_workspace_size(int64_t C, size_t* bytes);
/* Batch statistics of z [N, C]: stats (device float64 [2C + 1]) = [Σz | Σz² | N] — summable
 * across ranks (SyncBN: all-reduce them, then gnn_bn_finalize_f32).  finalize != 0 also does
 * gnn_bn_finalize_f32 in the same launch sequence (single device; with momentum >= 0 the merge
 * and the finalize are one launch). */
gnn_status gnn_bn_stats_f32(const float* z, int64_t ldz, int64_t N, int64_t C, double* stats, int32_t finalize,
                            float eps, float momentum, float* mean, float* invstd, float* running_mean,
                            float* running_var, int64_t* num_batches_tracked, void* workspace,
                            size_t workspace_bytes, gnn_stream_t stream);
/* mean = Σz/n, var = Σz²/n − mean² (biased, float64), invstd = 1/sqrt(var + eps); when
 * running_mean != NULL the nn.BatchNorm1d update: running = (1−m)·running + m·stat with the
 * unbiased variance, m = momentum (momentum < 0: PyTorch's momentum=None cumulative average
 * 1/(num_batches_tracked+1)), and num_batches_tracked += 1 (optional pointer). */
gnn_status gnn_bn_finalize_f32(const double* stats, int64_t C, float eps, float momentum, float* mean,
                               float* invstd, float* running_mean, float* running_var,
                               int64_t* num_batches_tracked, gnn_stream_t stream);
/* h = dropout(relu((z − mean)·invstd·weight + bias)) + r   (r optional; counter-hash dropout of
 * element r·C + c as gnn_agg_params; N·C < 2^32). */
gnn_status gnn_bn_act_res_fwd_f32(const float* z, int64_t ldz, const float* r, int64_t ldr, int64_t N, int64_t C,
                                  const float* mean, const float* invstd, const float* weight, const float* bias,
                                  float dropout_p, uint64_t seed, const int64_t* seed_ptr, float* h, int64_t ldh,
                                  gnn_stream_t stream);
/* Backward, step 1: sums (device float [2C]) = [Σ dy | Σ dy·x̂] over the N rows, with
 * dy = dh ⊙ dropout-mask/(1−p) ⊙ [y > 0] recomputed from z (the BN weight / bias gradients are
 * these local sums; SyncBN all-reduces a copy before step 2). */
gnn_status gnn_bn_act_bwd_reduce_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N,
                                     int64_t C, const float* mean, const float* invstd, const float* weight,
                                     const float* bias, float dropout_p, uint64_t seed, const int64_t* seed_ptr,
                                     float* sums, void* workspace, size_t workspace_bytes, gnn_stream_t stream);
/* Backward, step 2: dz = weight·invstd·(dy − Σdy/n − x̂·Σdy·x̂/n) with the (global) sums and the
 * device row count *n_total (stats[2C] of the forward; torch.batch_norm_backward_elemt). */
gnn_status gnn_bn_act_bwd_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N, int64_t C,
                              const float* mean, const float* invstd, const float* weight, const float* bias,
                              float dropout_p, uint64_t seed, const int64_t* seed_ptr, const float* sums,
                              const double* n_total, float* dz, int64_t lddz, gnn_stream_t stream);
/* The same, also writing the column sums of the dz it stores per block, colsum[b·C + c] for
 * b < gnn_bn_act_bwd_colsum_blocks(N, C) (N >= 1, C <= 256; ABI 21): the bias gradient of the
 * conv that produced z, through gnn_colsum_finish_f32, without a pass over dz. */
gnn_status gnn_bn_act_bwd_colsum_blocks(int64_t N, int64_t C, int32_t* nb);
gnn_status gnn_bn_act_bwd_colsum_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N, int64_t C,
                                     const float* mean, const float* invstd, const float* weight, const float* bias,
                                     float dropout_p, uint64_t seed, const int64_t* seed_ptr, const float* sums,
                                     const double* n_total, float* dz, int64_t lddz, float* colsum,
                                     gnn_stream_t stream);

/* K13: SAGEResBNNet's input with the fixed sinusoid time features, out = [x | te(t)] in one pass
 * (replaces SAGEResBN._time_embed / torch.cat of src/models/gnn.py:145-160, 172-176):
 * te_k = sin(t·2π(k+1)) for k < dim/2, cos(t·2π(k-dim/2+1)) for k < 2·(dim/2), 0 after, with
 * t = clamp(t_idx - 1, 0, T - 1) / max(T - 1, 1) (T = max_timestep).  x [N, F] (ldx), t_idx int64
 * [N], out [N, F + dim] (ldo).  No gradient: the features carry no parameters. */
gnn_status gnn_time_inject_sin_f32(const float* x, int64_t ldx, int64_t N, int64_t F, const int64_t* t_idx,
                                   int64_t dim, int64_t max_timestep, float* out, int64_t ldo, gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Step ops around the hot path (src/train_gnn.py:136-183, 201-206)          */
/* ------------------------------------------------------------------------ */
/* Masked class-weighted cross entropy over all N rows, forward and backward in one pass:
 * rows with mask[i] != 0 and 0 <= y[i] < C contribute loss_i = -w[y_i]·log_softmax(x_i)[y_i]
 * (F.cross_entropy(weight=w, reduction='none')); *loss = Σ loss_i · inv_denom (the reference's
 * loss_vec.mean() with inv_denom = 1 / n_train, src/train_gnn.py:175); dlogits = d(*loss)/dx
 * (zero on every other row).  C <= 16.  Deterministic fixed-order reduction. */
gnn_status gnn_masked_ce_workspace_size(int64_t N, size_t* bytes);
/* loss = NULL (ABI 18): the per-block partial sums stay in the workspace (its first ceil(N / 256)
 * floats) and the loss is finished later — by gnn_masked_ce_finish, or inside a gnn_clip_adam_f32
 * call (gnn_adam_group.loss_partial) when nothing reads it before the optimizer (a captured step). */
gnn_status gnn_masked_ce_finish(const float* partial, int32_t nblk, float inv_denom, float* loss, gnn_stream_t stream);
/* gnn_masked_ce_f32 (N >= 1) that also writes the per-256-row-block column sums of dlogits,
 * colsum[b * C + c], b < ceil(N / 256) (ABI 21): gnn_colsum_finish_f32(colsum, ceil(N / 256), C, db)
 * is then the output layer's bias gradient without a pass over dlogits. */
/* GCN's output layer and the masked CE in one launch (ABI 21): logits = Â·t + bias (gnn_aggregate_f32
 * GCN over a LOOPS_REPLACE plan, dinv = gnn_gcn_norm_f32, 1 <= C <= 2) and gnn_masked_ce_f32 of
 * them with its workspace contract (loss NULL: partials deferred); colsum (optional): the
 * per-256-row-block column sums of dlogits as gnn_masked_ce_colsum_f32 writes them. */
gnn_status gnn_gcn_out_ce_f32(const gnn_graph* g, const float* dinv, const float* t, int64_t ldt, int32_t C,
                              const float* bias, float* logits, int64_t ldo, const int64_t* y, const uint8_t* mask,
                              const float* class_w, float inv_denom, float* dlogits, int64_t ld_d, float* colsum,
                              float* loss, void* workspace, size_t workspace_bytes, gnn_stream_t stream);
gnn_status gnn_masked_ce_colsum_f32(int64_t N, int32_t C, const float* logits, int64_t ldx, const int64_t* y,
                                    const uint8_t* mask, const float* class_w, float inv_denom, float* dlogits,
                                    int64_t ld_d, float* loss, void* workspace, size_t workspace_bytes,
                                    float* colsum, gnn_stream_t stream);
gnn_status gnn_masked_ce_f32(int64_t N, int32_t C, const float* logits, int64_t ldx, const int64_t* y,
                             const uint8_t* mask, const float* class_w, float inv_denom, float* dlogits,
                             int64_t ld_d, float* loss, void* workspace, size_t workspace_bytes,
                             gnn_stream_t stream);

/* clip_grad_norm_(max_norm) + torch.optim.Adam.step() (weight_decay as L2 on the gradient) over
 * up to GNN_ADAM_MAX_TENSORS parameters (src/train_gnn.py:203-206).  `step` is a device float
 * incremented by the call (graph-replay safe); norm_out (optional, device) gets the pre-clip
 * total norm.  max_norm <= 0 disables clipping.  Grads are scaled in place, as torch does. */
#define GNN_ADAM_MAX_TENSORS 24
typedef struct {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq; int64_t numel;
} gnn_adam_tensor;
typedef struct {
  int32_t num_tensors;
  double lr, beta1, beta2, eps, weight_decay, max_norm;  /* double, as torch's Python scalars */
  gnn_adam_tensor tensors[GNN_ADAM_MAX_TENSORS];
  int32_t skip_nonfinite;  /* != 0: torch.amp.GradScaler.step semantics — any inf / NaN gradient
                              ELEMENT skips the update (params, moments, grads and step count
                              untouched); finite gradients whose Σg² overflows are clipped by
                              coefficient 0, as clip_grad_norm_ does with an inf norm */
  int64_t* bump_counter;   /* optional (ABI 18): a device int64 the call increments by one (the
                              dropout seed counter of a captured step — gnn_gemm_nt_params.seed_ptr
                              — advanced at the step's end instead of by a launch of its own) */
  const float* loss_partial; int32_t loss_nblk; float loss_scale; float* loss_out;
                           /* optional (ABI 18): *loss_out = loss_scale · Σ loss_partial[0 .. loss_nblk)
                              in gnn_masked_ce_f32's order — the loss of a gnn_masked_ce_f32 call made
                              with loss = NULL, finished in this call */
  const float* grad_sq_partial; int32_t grad_sq_nblk;
                           /* optional (ABI 20): the norm partials a gnn_gemm_tn_f32 call wrote
                              (gnn_gemm_tn_params.sq_partial, nb = grad_sq_nblk) for EXACTLY these
                              tensors' gradients, with *step as sq_step: the call then launches only the
                              clip + Adam kernel (its Σg² pass is folded into the TN's reduce) */
} gnn_adam_group;
/* Workspace: 2·64 + 2 words, ZEROED before the first call.  Without grad_sq_partial, gradients of
 * at most 2^15 elements in all (GCN, GAT of the path) run as ONE launch: each block sums Σg² over
 * all of them itself, in one fixed order, and the last block to finish advances *step (a vector
 * atomic on the workspace's last word, a running count: each call adds exactly 64 and the block
 * that draws 63 mod 64 is the last, so a call that never completed cannot leave later calls
 * without a last block — no reset is needed, re-zeroing the workspace is always safe between
 * calls); larger ones run the Σg² pass first (two launches).  ABI 21. */
gnn_status gnn_clip_adam_workspace_size(size_t* bytes);
gnn_status gnn_clip_adam_f32(const gnn_adam_group* group, float* step, float* norm_out, void* workspace,
                             size_t workspace_bytes, gnn_stream_t stream);

/* ------------------------------------------------------------------------ */
/* K11 NeighborLoader neighbour sampling (torch_geometric.loader.NeighborLoader + pyg-lib
 *     neighbor_sample, built at src/train_gnn.py:329-348 and consumed by
 *     train_epoch_minibatch / eval_val_minibatch, src/train_gnn.py:212-276)            */
/* ------------------------------------------------------------------------ */
/* Workspace for gnn_neighbor_sample over a graph of num_nodes with the given capacities. */
gnn_status gnn_neighbor_sample_workspace_size(int64_t num_nodes, int64_t node_cap, int64_t edge_cap,
                                              size_t* bytes);

/* Sample one batch over the CSR-by-target direction of `g` (a GNN_LOOPS_KEEP plan of the
 * full graph's edge_index): seeds[num_seeds] (distinct, device int32) become local nodes
 * 0..B-1; hop h samples up to fanout[h] (host array; -1 = all, else >= 1) in-neighbours of
 * every node first discovered in hop h-1, uniformly without replacement (all of them when the
 * in-degree is <= fanout), from a counter hash of (seed, hop, node, draw).  New nodes are
 * appended to n_id in order of first appearance in the hop's edge list (disjoint=False dedup).
 * Edges: e_src[s] -> e_dst[s] in local ids (the original edge direction), e_id[s] = PyG edge
 * id (csr_eid[slot], or the CSR slot when csr_eid is NULL); hop-major, then frontier node,
 * then PyG edge order.  hop_nodes[num_hops+1] / hop_edges[num_hops] (HOST arrays) receive
 * PyG's num_sampled_nodes / num_sampled_edges.  Output sizes are data dependent: the call
 * synchronises `stream` twice per hop to read them.  INVALID_ARG when a capacity is exceeded
 * or seeds repeat, INDEX_OUT_OF_RANGE for a seed outside [0, N). */
gnn_status gnn_neighbor_sample(const gnn_graph* g, const int32_t* csr_eid, const int32_t* seeds,
                               int64_t num_seeds, int32_t num_hops, const int32_t* fanout, uint64_t seed,
                               int32_t* n_id, int64_t node_cap, int32_t* e_src, int32_t* e_dst,
                               int32_t* e_id, int64_t edge_cap, int64_t* hop_nodes, int64_t* hop_edges,
                               void* workspace, size_t workspace_bytes, gnn_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GNNMP_H_ */
