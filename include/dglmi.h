/*
 * dglmi.h -- C ABI of the MI355X-native g-SpMM / g-SDDMM engine.
 *
 * Drop-in boundary for the reference's kernel FFI.  The reference exposes
 * its hot path as DGL PackedFuncs registered in src/kernel/binary_reduce.cc
 * and bound by python/dgl/kernel.py through ctypes; every entry point below
 * names the PackedFunc it replaces.  Arguments are plain pointers and sizes:
 * graphs are raw CSR arrays, tensors are (pointer, ndim, shape) records of
 * contiguous row-major fp32 device memory, streams are hipStream_t passed as
 * void* (NULL = the default stream).
 *
 * Conventions shared with the reference:
 *   - target codes: 0 = src, 1 = dst, 2 = edge, 3 = none
 *     (binary_reduce_common.h:39-44, function/base.py:13-15);
 *   - reducer strings "sum" | "max" | "min" | "prod" | "none"; "mean" is
 *     rejected exactly like the reference C++ (binary_reduce_impl.h:95-98):
 *     the Python layer divides by the degree (tensor.py:308-325);
 *   - op strings "add" | "sub" | "mul" | "div" | "dot" | "use_lhs";
 *   - outputs are OVERWRITTEN completely (identity fill then reduce,
 *     binary_reduce_impl.h:31-64); gradients likewise (zero fill, :119-160);
 *   - errors: every function returns 0 on success and -1 on failure, with the
 *     message available from DGLMIGetLastError() in thread-local storage
 *     (runtime_base.h:13-32, c_runtime_api.cc:138-148).  Nothing calls exit().
 *
 * Deliberate differences (documented in DESIGN.md):
 *   - device work only (gfx950); fp32 features; int32 indices -- the same
 *     envelope as the reference GPU path (common.h:49-69) -- or, for graphs of
 *     2^31 or more edges (num_bits == 64), int64 offsets and edge ids with int32
 *     node ids, where the reference falls back to its int64 CPU kernels
 *     (graph_index.py:941-952, cpu/binary_reduce_sum.cc:15-23);
 *   - an edge-target mapping is indexed by edge id (the value of csr.data),
 *     not by CSR position, so one mapping serves every traversal direction;
 *   - node mappings (src/dst targets) must be injective (they are relabel
 *     maps in the reference, spmv.py:126-180) because reductions are
 *     owner-computes (one writer per output row, no atomics).
 */
#ifndef DGLMI_H_
#define DGLMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGLMI_MAX_NDIM 8

enum DGLMITarget {
  DGLMI_TARGET_SRC = 0,
  DGLMI_TARGET_DST = 1,
  DGLMI_TARGET_EDGE = 2,
  DGLMI_TARGET_NONE = 3
};

/* One direction of the adjacency (aten::CSRMatrix, include/dgl/array.h).
 * When the graph's num_bits is 64, `indptr` and `data` point at int64_t arrays
 * (cast the pointers); indices and rows are int32 in both layouts. */
typedef struct {
  int64_t num_rows;
  int64_t num_cols;
  int64_t nnz;
  const int32_t* indptr;  /* num_rows + 1 (int64 values when num_bits == 64) */
  const int32_t* indices; /* nnz, column node ids */
  const int32_t* data;    /* nnz, edge ids (int64 values when num_bits == 64) */
  const int32_t* rows;    /* nnz, row id of every position (COO rows, ascending);
                             required: the edge-wise kernels and the load-balanced
                             reduce path read the row of a position from it */
} DGLMICsr;

/* ImmutableGraph as the kernels see it (csr_interface.h:23-29). */
typedef struct {
  DGLMICsr in_csr;        /* rows = destination nodes, cols = source nodes */
  DGLMICsr out_csr;       /* rows = source nodes, cols = destination nodes */
  int32_t num_bits;       /* 32, or 64: int64 indptr / data (graphs of >= 2^31 edges;
                             node ids < 2^31).  64-bit graphs take every builtin
                             message / reduce / SDDMM / edge-softmax entry without
                             mappings; the fused GAT, R-GCN, NbAccess, partitioning
                             and column-block entries need 32. */
  int32_t device;         /* HIP device ordinal the arrays live on */
  void* workspace;        /* caller-owned scratch for this call (may be NULL) */
  int64_t workspace_bytes;
  /* Optional edge list in edge-id order (ImmutableGraph's COO, immutable_graph.h):
   * coo_src[e], coo_dst[e] for e in [0, in_csr.nnz).  Only valid when in_csr.data
   * is a permutation of [0, nnz) (whole graphs, not parent-eid subgraphs).  When
   * present, per-edge outputs (reducer "none", edge gradients) are produced in
   * edge-id order: sequential writes and edge-operand reads.  May be NULL. */
  const int32_t* coo_src;
  const int32_t* coo_dst;
  /* Optional cache-placement hints (extension, no reference counterpart):
   * in_csr.indices / out_csr.indices with bit 31 set on every column whose
   * node row is gathered fewer than `min_hot_degree` times per pass over that
   * CSR (DGLMIKernelMarkColdColumns).  When present and the gathered table
   * exceeds the 256 MiB Infinity Cache, the copy_u sum kernels load marked rows
   * non-temporally so that rarely re-read rows do not evict the re-read ones
   * from L2 / Infinity Cache (M1: 3.24 -> 3.11 ms per copy_u_sum, bit-identical
   * results).  Either may be NULL. */
  const int32_t* in_gather_cols;
  const int32_t* out_gather_cols;
  /* Optional column blocks (extension, no reference counterpart): when
   * num_col_blocks > 1, in_col_blocks[b] holds the positions of in_csr whose
   * source lies in the b-th of num_col_blocks equal node-id ranges and
   * out_col_blocks[b] the positions of out_csr whose destination lies in the
   * b-th range -- each a full-height CSR (same num_rows / num_cols, rows keep
   * their positions' original order, `data` = edge ids, `rows` required).  The
   * fused GAT kernels then run one launch per block, so the rows gathered by a
   * launch fit the 4 MiB per-XCD L2 better, and merge the per-block softmax
   * partials (forward) or accumulate the gradients (backward) in block order.
   * C3 (Reddit-size, 8 blocks): forward 5.54 -> ~4 ms.  NULL / 0 = off. */
  int32_t num_col_blocks;
  const DGLMICsr* in_col_blocks;
  const DGLMICsr* out_col_blocks;
  /* Optional per-graph R-GCN state (extension): built once by DGLMIRgcnPrepare and
   * read by the DGLMIRgcnLayer* entries when it matches the graph's etypes (and the
   * call's norm) pointers.  NULL = every call derives what it needs from etypes / norm. */
  const struct DGLMIRgcnState* rgcn;
  /* Optional (extension): for every in-CSR position p, the out-CSR position of the
   * same edge.  When present and the fused GAT backward runs unblocked (no column
   * blocks), it drops its destination-side walk: the source-side walk stores each
   * edge's grad_er term in out-CSR order and grad_er is one gather-sum over the
   * in-CSR (a 256-B feature row and a logit gathered per edge become one H-float
   * term; C3 unblocked 11.98 -> 9.57 ms).  NULL = the destination-side walk. */
  const int32_t* gat_edge_pos;
  /* Optional relation id of every edge (the hack's typed edges: Graph::AddEdgesWithType
   * stores them in the graph object and the R-GCN kernels read them from there through
   * GetCsrSortedByEdgeType, src/graph/graph.cc:690-746, binary_reduce_impl.cu:951,1020,
   * 1128,1208).  One int32 per edge id, each in [0, num_rels) where num_rels is the
   * weight's leading dimension.  Read only by the DGLMIRgcn* entries, which therefore
   * keep the reference's argument lists.  NULL for untyped graphs. */
  const int32_t* etypes;
  /* Optional (extension): bit 0 set when in_csr.data[p] == p for every position p,
   * bit 1 the same for out_csr -- a view whose edge ids are one walk's positions, with
   * per-edge operands permuted into that order (dgl's position_view).  The
   * load-balanced reduce then takes edge p's operand at p without streaming `data`, and
   * a per-edge scalar operand is staged with the walk's rows and columns instead of
   * gathered per lane.  0 = read `data`. */
  int32_t eid_identity;
} DGLMIGraph;

/* A contiguous row-major fp32 device array (NDArray / DLTensor subset). */
typedef struct {
  float* data;
  int32_t ndim;
  int64_t shape[DGLMI_MAX_NDIM + 1];
} DGLMIArray;

/* Optional epilogue fused into a "sum" reduction (extension): every output
 * row r becomes (((out[r] * row_mul[r]) / row_div[r]) + bias) + addend[r],
 * applied once to the finished row, in that order -- GraphConv's `rst * norm`
 * then `+ bias` (graphconv.py:158-170), the mean reducer's `out / degs`
 * (tensor.py:308-325), and accumulation onto an earlier partial result (the
 * halo half of a partitioned aggregation) -- without extra passes over the
 * output.  Any pointer may be NULL; row_mul / row_div have one float per output
 * row, bias one per output feature, addend the output's shape (it must not
 * overlap the output: rows split across work chunks keep partial sums there). */
typedef struct {
  const float* row_mul;
  const float* row_div;
  const float* bias;
  const float* addend;
} DGLMIEpilogue;

/* Last error message of the calling thread (DGLGetLastError). */
const char* DGLMIGetLastError(void);

/* Library version string ("0.4-mi355x"). */
const char* DGLMIVersion(void);

/* Item order of the per-edge (g-SDDMM) kernels, process-wide (extension, no
 * reference counterpart).  AUTO (the default) picks edge-id order or in-CSR
 * order per call from the operand shapes and the graph's average degree
 * (DESIGN.md 4.2b); COO / CSR force one, so tests cover both walks. */
enum DGLMISddmmOrder {
  DGLMI_SDDMM_ORDER_AUTO = 0,
  DGLMI_SDDMM_ORDER_COO = 1,
  DGLMI_SDDMM_ORDER_CSR = 2
};
int DGLMISetSddmmOrder(int32_t order);

/* _CAPI_DGLKernelInferBinaryFeatureShape (binary_reduce.cc:281-293).
 * Writes the broadcast feature shape into out_shape (capacity
 * DGLMI_MAX_NDIM + 1) and its rank into *out_ndim. Host-only. */
int DGLMIKernelInferBinaryFeatureShape(const char* op, const DGLMIArray* lhs,
                                       const DGLMIArray* rhs, int64_t* out_shape,
                                       int32_t* out_ndim);

/* _CAPI_DGLKernelBinaryOpReduce (binary_reduce.cc:357-378). */
int DGLMIKernelBinaryOpReduce(const char* reducer, const char* op, const DGLMIGraph* graph,
                              int32_t lhs_target, int32_t rhs_target,
                              const DGLMIArray* lhs, const DGLMIArray* rhs, DGLMIArray* out,
                              const int32_t* lhs_mapping, const int32_t* rhs_mapping,
                              const int32_t* out_mapping, void* stream);

/* _CAPI_DGLKernelBackwardLhsBinaryOpReduce (binary_reduce.cc:502-527). */
int DGLMIKernelBackwardLhsBinaryOpReduce(
    const char* reducer, const char* op, const DGLMIGraph* graph, int32_t lhs_target,
    int32_t rhs_target, const int32_t* lhs_mapping, const int32_t* rhs_mapping,
    const int32_t* out_mapping, const DGLMIArray* lhs, const DGLMIArray* rhs,
    const DGLMIArray* out, const DGLMIArray* grad_out, DGLMIArray* grad_lhs, void* stream);

/* _CAPI_DGLKernelBackwardRhsBinaryOpReduce (binary_reduce.cc:600-626). */
int DGLMIKernelBackwardRhsBinaryOpReduce(
    const char* reducer, const char* op, const DGLMIGraph* graph, int32_t lhs_target,
    int32_t rhs_target, const int32_t* lhs_mapping, const int32_t* rhs_mapping,
    const int32_t* out_mapping, const DGLMIArray* lhs, const DGLMIArray* rhs,
    const DGLMIArray* out, const DGLMIArray* grad_out, DGLMIArray* grad_rhs, void* stream);

/* _CAPI_DGLKernelCopyReduce (binary_reduce.cc:649-665). */
int DGLMIKernelCopyReduce(const char* reducer, const DGLMIGraph* graph, int32_t target,
                          const DGLMIArray* in, DGLMIArray* out, const int32_t* in_mapping,
                          const int32_t* out_mapping, void* stream);

/* DGLMIKernelBinaryOpReduce / DGLMIKernelCopyReduce with a fused epilogue
 * (reducer must be "sum"; epilogue may be NULL). */
int DGLMIKernelBinaryOpReduceEx(const char* reducer, const char* op, const DGLMIGraph* graph,
                                int32_t lhs_target, int32_t rhs_target,
                                const DGLMIArray* lhs, const DGLMIArray* rhs, DGLMIArray* out,
                                const int32_t* lhs_mapping, const int32_t* rhs_mapping,
                                const int32_t* out_mapping, const DGLMIEpilogue* epilogue,
                                void* stream);
int DGLMIKernelCopyReduceEx(const char* reducer, const DGLMIGraph* graph, int32_t target,
                            const DGLMIArray* in, DGLMIArray* out, const int32_t* in_mapping,
                            const int32_t* out_mapping, const DGLMIEpilogue* epilogue,
                            void* stream);

/* _CAPI_DGLKernelBackwardCopyReduce (binary_reduce.cc:697-716). */
int DGLMIKernelBackwardCopyReduce(const char* reducer, const DGLMIGraph* graph, int32_t target,
                                  const DGLMIArray* in, const DGLMIArray* out,
                                  const DGLMIArray* grad_out, DGLMIArray* grad_in,
                                  const int32_t* in_mapping, const int32_t* out_mapping,
                                  void* stream);

/* Bytes of DGLMIGraph.workspace a reduce-to-node call over `csr` with
 * feature length `feat_len` needs on the load-balanced path (0 if none).
 * The load-balanced path cuts the CSR positions into fixed-size edge chunks
 * (no reference counterpart: the reference relies on minigun's per-edge
 * binary search, binary_reduce_impl.cu:424-466); rows split across chunks
 * leave per-chunk partials here, combined afterwards in chunk order (rows of
 * more than 32 continuation chunks in segments of 32, in segment order), plus
 * one int32 counter per chunk for those segmented rows. */
int64_t DGLMIKernelWorkspaceBytes(const DGLMICsr* csr, int64_t feat_len);

/* Build DGLMIGraph.{in,out}_gather_cols (extension): out_cols[p] =
 * csr.indices[p] | (1 << 31) when the column node's row count in the opposite
 * direction (out-degree of a source for the in-CSR, in-degree of a destination
 * for the out-CSR) is below min_hot_degree, else csr.indices[p].  `direction`
 * 0 marks the in-CSR, 1 the out-CSR; out_cols is a device array of csr.nnz
 * int32.  Stream-ordered. */
int DGLMIKernelMarkColdColumns(const DGLMIGraph* graph, int32_t direction,
                               int32_t min_hot_degree, int32_t* out_cols, void* stream);

/* ---- graph ingestion ------------------------------------------------------
 * aten::COOToCSR (array/cpu/spmat_op_impl_coo.cc:230-283): stable counting
 * sort by row, data = original position (or data[i] when given).  Host
 * arrays, int64 (the reference's IdArray width for mutable graphs). */
int DGLMICOOToCSR(int64_t num_rows, int64_t nnz, const int64_t* row, const int64_t* col,
                  const int64_t* data, int64_t* indptr, int64_t* indices, int64_t* out_data);
/* aten::CSRTranspose (array/cpu/spmat_op_impl.cc:323-369). Host, int64. */
int DGLMICSRTranspose(int64_t num_rows, int64_t num_cols, const int64_t* indptr,
                      const int64_t* indices, const int64_t* data, int64_t* t_indptr,
                      int64_t* t_indices, int64_t* t_data);
/* Device COO -> CSR (int32), bit-identical to DGLMICOOToCSR: a stable
 * counting sort by row on the GPU.  All pointers are device memory;
 * `workspace` must hold DGLMICOOToCSRDeviceWorkspaceBytes(num_rows, nnz). */
int64_t DGLMICOOToCSRDeviceWorkspaceBytes(int64_t num_rows, int64_t nnz);
int DGLMICOOToCSRDevice(int64_t num_rows, int64_t nnz, const int32_t* row, const int32_t* col,
                        const int32_t* data, int32_t* indptr, int32_t* indices,
                        int32_t* out_data, void* workspace, int64_t workspace_bytes,
                        void* stream);
/* Row id of every CSR position (CSRToCOO rows, spmat_op_impl.cc:375-387), device. */
int DGLMICSRExpandRows(const int32_t* indptr, int64_t num_rows, int64_t nnz, int32_t* rows,
                       void* stream);
/* 64-bit graphs (num_bits == 64): device COO -> CSR with int64 offsets and edge ids
 * (row / col int32 node ids, optional int64 data; indptr int64, indices int32,
 * out_data int64), bit-identical to DGLMICOOToCSR; a stable counting sort in
 * batches of 2^30 positions.  Workspace: DGLMICOOToCSRDevice64WorkspaceBytes. */
int64_t DGLMICOOToCSRDevice64WorkspaceBytes(int64_t num_rows, int64_t nnz);
int DGLMICOOToCSRDevice64(int64_t num_rows, int64_t nnz, const int32_t* row, const int32_t* col,
                          const int64_t* data, int64_t* indptr, int32_t* indices,
                          int64_t* out_data, void* workspace, int64_t workspace_bytes,
                          void* stream);
/* DGLMICSRExpandRows for an int64 indptr. */
int DGLMICSRExpandRows64(const int64_t* indptr, int64_t num_rows, int64_t nnz, int32_t* rows,
                         void* stream);

/* ---- fused GAT (hack kernels _CAPI_DGLFusedGatKernel / _CAPI_DGLKernelBackwardFusedGat,
 * binary_reduce.cc:380-396, 529-549) ------------------------------------------
 * out[v,h,:] = sum_{u->v} softmax_v(leaky(el[u,h] + er[v,h])) * feat_src[u,h,:], with a
 * max-stabilised online softmax; instead of the reference's per-edge exp[E,H] and
 * sum[N,H] buffers the forward keeps max_out[N,H] and sum_out[N,H] (= sum exp(s - max)).
 * feat_src (N_src, H, D) with D a multiple of 4 and D/4 a power of two, H*D <= 1024;
 * el (N_src, H[, 1]); er (N_dst, H[, 1]); out (N_dst, H, D).  The backward writes all
 * three gradients (overwriting). */
int DGLMIFusedGatForward(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                         const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                         DGLMIArray* max_out, DGLMIArray* sum_out, void* stream);
int DGLMIFusedGatBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                          const DGLMIArray* er, float negative_slope, const DGLMIArray* out,
                          const DGLMIArray* max_in, const DGLMIArray* sum_in,
                          const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                          DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream);
/* Extension: the forward also keeps, per destination row v and head h, the slope
 * aggregates of the attention (lrelu' = 1 where the logit's pre-activation el + er is
 * positive, else the negative slope):
 *   slope_sum[v, h]     = sum_{e into v} a_e * lrelu'(pre_e)                 (N_dst, H)
 *   slope_feat[v, h, :] = sum_{e into v} a_e * lrelu'(pre_e) * feat_src[u, h, :]  (N_dst, H, D)
 * (16-byte aligned), one more running sum beside the output's.  Handed to
 * DGLMIFusedGatBackwardEx they give grad_er[v, h] = <grad_out[v, h], slope_feat[v, h]>
 * - delta[v, h] * slope_sum[v, h] (delta = <grad_out[v, h], out[v, h]>) from one dense
 * pass: the backward runs only the source-side walk over the out-CSR. */
int DGLMIFusedGatForwardEx(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                           const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                           DGLMIArray* max_out, DGLMIArray* sum_out, DGLMIArray* slope_feat,
                           DGLMIArray* slope_sum, void* stream);
int DGLMIFusedGatBackwardEx(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                            const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                            const DGLMIArray* out, const DGLMIArray* max_in,
                            const DGLMIArray* sum_in, const DGLMIArray* slope_feat,
                            const DGLMIArray* slope_sum, const DGLMIArray* grad_out,
                            DGLMIArray* grad_feat_src, DGLMIArray* grad_el, DGLMIArray* grad_er,
                            void* stream);

/* Fused GAT with attention dropout (GATConv's attn_drop in training, gatconv.py:154:
 * dropout on the softmax weights, per edge and head).  Edge e, head h keeps its weight,
 * when a counter hash of (seed, e) -- one key per edge, one more mix per pair of heads,
 * 16 bits per head -- clears the threshold t = round(attn_drop * 2^16) -- a mask no buffer
 * holds: the backward recomputes it from the same seed and the walks' edge ids.  Kept
 * weights are scaled by 2^16 / (2^16 - t), the inverse of the quantised keep probability
 * (within 2^-17 of 1 / (1 - attn_drop)); attn_drop in [0, 1], and t = 2^16 (attn_drop >=
 * 1 - 2^-17) drops every weight.  The softmax denominator (sum_out) is the plain
 * one; out and slope_feat carry the kept, rescaled weights.  The backward needs the
 * forward's slope aggregates.  attn_drop = 0 equals DGLMIFusedGatForwardEx /
 * BackwardEx bit for bit.  Extension: the reference has no fused dropout (its
 * FusedGATConv runs without one; GATConv composes dropout between edge_softmax and
 * u_mul_e_sum). */
int DGLMIFusedGatDropoutForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                                float attn_drop, uint64_t seed, DGLMIArray* out, DGLMIArray* max_out,
                                DGLMIArray* sum_out, DGLMIArray* slope_feat, DGLMIArray* slope_sum,
                                void* stream);
int DGLMIFusedGatDropoutBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                 const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                                 float attn_drop, uint64_t seed, const DGLMIArray* out,
                                 const DGLMIArray* max_in, const DGLMIArray* sum_in,
                                 const DGLMIArray* slope_feat, const DGLMIArray* slope_sum,
                                 const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                                 DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream);
/* Fused GAT with the CALLER's attention-dropout mask: keep holds one word of keep_bits
 * bits (8, 16 or 32; >= H) per edge (E = in_csr.nnz words), bit h set when head h keeps
 * its weight, and kept weights are scaled by keep_scale.  GATConv draws the mask with its
 * own nn.Dropout on an (E, H, 1) tensor of ones in edge-id order -- the draws the
 * reference's dropout(edge_softmax(...)) makes under the same seed (gatconv.py:154) --
 * packs it with DGLMIGatKeepBits into the narrowest word that holds H and passes
 * keep_scale = the dropout's 1 / (1 - p).  keep_by_position = 0: words indexed by edge id
 * (the walks read each through their CSR's edge ids, a random read per edge);
 * keep_by_position = 1: words in the walks' position order (DGLMIGatKeepGather by the
 * walk CSR's edge ids, once per direction): the forward's in-CSR (its column blocks
 * concatenated in block order when the graph carries them), the backward's out-CSR
 * (likewise) -- every read coalesced.  Otherwise as DGLMIFusedGatDropout*.  Extension. */
int DGLMIFusedGatKeepForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                             const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                             const void* keep, int keep_bits, int keep_by_position, float keep_scale,
                             DGLMIArray* out, DGLMIArray* max_out, DGLMIArray* sum_out,
                             DGLMIArray* slope_feat, DGLMIArray* slope_sum, void* stream);
int DGLMIFusedGatKeepBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                              const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                              const void* keep, int keep_bits, int keep_by_position, float keep_scale,
                              const DGLMIArray* out, const DGLMIArray* max_in, const DGLMIArray* sum_in,
                              const DGLMIArray* slope_feat, const DGLMIArray* slope_sum,
                              const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                              DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream);
/* torch's fused dropout draw over a contiguous (E, H) tensor, as the generator and the
 * launch left it: seed, offset (the generator's Philox offset before the draw, a multiple
 * of 4), threads = the dropout kernel's grid x 256 (grid = min(ceil(E H / 256), CUs x
 * maxThreadsPerCU / 256)), vec = 4 / 2 / 1 (E H divisible by 4 / by 2 / neither), keep =
 * float(1 - p), scale = the kept weights' factor (float(1 / float(1 - p))).  Element i is
 * kept when the Philox4x32-10 uniform the kernel drew for it is below keep (internal.h
 * dropout_draw_slot; scripts/philox_probe.py pins the mapping on this build). */
typedef struct {
  uint64_t seed;
  uint64_t offset;
  int64_t threads;
  int32_t vec;
  float keep;
  float scale;
} DGLMIDropoutDraw;
/* Fused GAT with torch's own attention-dropout draws recomputed inside the walks: edge e,
 * head h keeps its weight (scaled by draw->scale) when the draw keeps element e * H + h
 * of the (E, H) attention tensor in edge-id order -- what nn.Dropout(p) draws on the
 * reference's dropout(edge_softmax(...)) (gatconv.py:154) from the same generator state.
 * No mask in memory, nothing gathered; GATConv advances the generator as the draw would.
 * Otherwise as DGLMIFusedGatKeep*.  Extension. */
int DGLMIFusedGatDrawForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                             const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                             const DGLMIDropoutDraw* draw, DGLMIArray* out, DGLMIArray* max_out,
                             DGLMIArray* sum_out, DGLMIArray* slope_feat, DGLMIArray* slope_sum, void* stream);
int DGLMIFusedGatDrawBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                              const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                              const DGLMIDropoutDraw* draw, const DGLMIArray* out, const DGLMIArray* max_in,
                              const DGLMIArray* sum_in, const DGLMIArray* slope_feat,
                              const DGLMIArray* slope_sum, const DGLMIArray* grad_out,
                              DGLMIArray* grad_feat_src, DGLMIArray* grad_el, DGLMIArray* grad_er,
                              void* stream);
/* mask[i] = 1 if the draw keeps element i, else 0, for i < n (n % vec == 0): the whole
 * mask of the draw above (the fused route's self-check against torch.native_dropout, and
 * the tests).  Extension. */
int DGLMIDropoutDrawMask(const DGLMIDropoutDraw* draw, int64_t n, uint8_t* mask, void* stream);
/* out[p * heads + h] = draw->scale if the draw keeps element eids[p] * heads + h, else 0,
 * for p < n (eids NULL = identity; heads <= 32; n = the draw's E): nn.Dropout's output on
 * an (E, heads) tensor of ones, in a walk's position order -- GATConv's composition on its
 * position view multiplies the attention by it.  Extension. */
int DGLMIDropoutDrawScale(const DGLMIDropoutDraw* draw, int heads, const int32_t* eids, int64_t n, float* out,
                          void* stream);
/* x[p * heads + h] *= that factor, in place: dropout(x) on a walk-ordered (E, heads) tensor
 * with the draws of edge eids[p] (one read and one write of x instead of the factor's
 * write plus a separate multiply).  Extension. */
int DGLMIDropoutDrawApply(const DGLMIDropoutDraw* draw, int heads, const int32_t* eids, int64_t n, float* x,
                          void* stream);
/* out[i] = keep[index[i]] for i < n, words of keep_bits bits (8, 16, 32): keep words in
 * edge-id order into a walk's position order (index = that CSR's edge ids, int32).
 * Device pointers; indices must lie in range.  Extension. */
int DGLMIGatKeepGather(const void* keep, int keep_bits, const int32_t* index, int64_t n, void* out,
                       void* stream);
/* bits[e] = OR over h < heads of (table[e * heads + h] != 0) << h for e < num_edges, in
 * words of keep_bits bits (8, 16 or 32; heads <= keep_bits): a dropout output (E, H)
 * packed to the keep words above.  Device pointers.  Extension. */
int DGLMIGatKeepBits(const float* table, int64_t num_edges, int heads, void* bits, int keep_bits,
                     void* stream);
/* The same from the dropout's boolean mask (E, H) bytes, non-zero = kept -- the second
 * output of torch.native_dropout, which nn.Dropout's fused path draws identically
 * (GATConv's default: a quarter of the table's bytes).  heads = 8 needs mask 8-byte
 * aligned.  Extension. */
int DGLMIGatKeepBitsMask(const uint8_t* mask, int64_t num_edges, int heads, void* bits, int keep_bits,
                         void* stream);
/* The same two kernels in the reference's argument order, for a binding of the hack's
 * PackedFuncs that keeps its Python caller unchanged (tensor.py:383-420):
 *   _CAPI_DGLFusedGatKernel(G, feat_src, el, er, sum, exp, ret, slope)
 *   _CAPI_DGLKernelBackwardFusedGat(G, feat_src, el, er, sum, exp, ret, grad_out,
 *                                   grad_feat_src, grad_el, grad_er, slope)
 * (binary_reduce.cc:380-396, 529-549).  sum (N_dst, H[, 1]) and exp (E, H[, 1]) are
 * caller-allocated state passed from the forward to the backward unchanged; their
 * contents are this library's softmax state, not the hack's per-edge exponentials:
 * when E >= N_dst, exp's first N_dst * H floats keep the running max and sum the sum
 * of exp(s - max) (bit-identical to DGLMIFusedGatForward / Backward), and when also
 * E >= about N_dst * (D + 2) (a 16-byte aligned exp), the slope aggregates of
 * DGLMIFusedGatForwardEx follow the max in exp (from float round_up(N_dst * H, 4)) and
 * the backward skips its destination-side walk; otherwise sum keeps max + log(sum)
 * and exp is not touched.  ret (N_dst, H, D) is overwritten, and
 * the three gradients are overwritten (the hack's caller zero-fills them first). */
int DGLMIFusedGatKernel(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                        const DGLMIArray* er, DGLMIArray* sum, DGLMIArray* exp, DGLMIArray* ret,
                        float slope, void* stream);
int DGLMIKernelBackwardFusedGat(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                const DGLMIArray* el, const DGLMIArray* er, const DGLMIArray* sum,
                                const DGLMIArray* exp, const DGLMIArray* ret,
                                const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                                DGLMIArray* grad_el, DGLMIArray* grad_er, float slope,
                                void* stream);
/* 1 if the fused GAT kernels support (heads, head_dim), else 0. */
int DGLMIFusedGatSupported(int64_t heads, int64_t head_dim);

/* Fused edge softmax over the in-edges of every destination node (extension:
 * the reference composes it from five kernels in Python,
 * python/dgl/nn/pytorch/softmax.py:15-114; same math, max-stabilised).
 * logits / out / grads: (E, ...) by edge id with H values per edge
 * (DGLMIEdgeSoftmaxSupported(H)).  The call needs
 * DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H) bytes of scratch, taken from
 * graph->workspace when it is large enough (else stream-ordered allocation). */
int DGLMIEdgeSoftmaxSupported(int64_t values_per_edge);
int64_t DGLMIEdgeSoftmaxWorkspaceBytes(const DGLMICsr* in_csr, int64_t values_per_edge);
int DGLMIEdgeSoftmaxForward(const DGLMIGraph* graph, const DGLMIArray* logits, DGLMIArray* out,
                            void* stream);
/* grad_logits = out * grad_out - out * sum_{in-edges}(out * grad_out) (softmax.py:86-114). */
int DGLMIEdgeSoftmaxBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                             const DGLMIArray* grad_out, DGLMIArray* grad_logits, void* stream);
/* GATConv's leaky_relu -> edge_softmax pair (gatconv.py:160-161) in the same passes
 * (extension): out = edge_softmax(leaky_relu(logits, negative_slope)), and
 * grad_logits = leaky_relu'(logits) * (the softmax backward of out, grad_out) with
 * leaky_relu'(x) = x > 0 ? 1 : negative_slope -- torch's leaky_relu /
 * leaky_relu_backward operations, so the results are those of the two-step form bit for
 * bit.  `logits` is the pre-activation input in both calls; the activated logits are
 * never written. */
/* GATConv's u_add_v -> leaky_relu -> edge_softmax chain (gatconv.py:158-161) with the
 * logits never stored (extension): the logit of edge (u -> v) is el[u] + er[v] (H values,
 * added as the u_add_v SDDMM adds them), computed where the softmax reads it; out =
 * edge_softmax(leaky_relu(el[u] + er[v])), and the backward writes the gradient wrt the
 * logits (before leaky_relu), the two-step forms' bits.  el: one row per source
 * (in_csr.num_cols), er: one row per destination; `out` / grads by edge id. */
int DGLMIEdgeSoftmaxNodeLogitsForward(const DGLMIGraph* graph, const DGLMIArray* el,
                                      const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                                      void* stream);
/* DGLMIEdgeSoftmaxNodeLogitsForward that also returns each destination row's softmax
 * statistics: row_max (N_dst, H) the maximum of its (activated) logits, row_sum (N_dst,
 * H) the sum of exp(logit - max) -- the state the fused GAT backward entries take as
 * max_in / sum_in, so GATConv's unfused composition can hand its backward to them
 * (rows without in-edges: left as the caller initialised them).  Extension. */
int DGLMIEdgeSoftmaxNodeLogitsForwardEx(const DGLMIGraph* graph, const DGLMIArray* el,
                                        const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                                        DGLMIArray* row_max, DGLMIArray* row_sum, void* stream);
int DGLMIEdgeSoftmaxNodeLogitsBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                                       const DGLMIArray* grad_out, const DGLMIArray* el,
                                       const DGLMIArray* er, float negative_slope,
                                       DGLMIArray* grad_logits, void* stream);
/* The bracketing projection Y = X W (+ bias) of GraphConv / GATConv / RelGraphConv
 * (torch.matmul in the reference, graphconv.py:146-170, gatconv.py:127-132) on MFMA, for
 * tall-skinny shapes: x (m, k) row-major, w (w_rows, n) element (i, j) at w[i *
 * w_stride_k + j * w_stride_n] (a transposed nn.Linear weight is strides (1, k)), bias
 * (n) or NULL, y (m, n) row-major; device pointers on `device`, x / y / bias 16-byte
 * aligned.  w_rows must equal k (a mismatch is an error, as torch.matmul's).
 * DGLMIProjectSupported(k, n): 1 <= k <= 640, 1 <= n <= 2^20 (extension). */
int DGLMIProjectSupported(int64_t k, int64_t n);
int DGLMIProject(const float* x, int64_t m, int64_t k, const float* w, int64_t w_rows,
                 int64_t w_stride_k, int64_t w_stride_n, int64_t n, const float* bias, float* y,
                 int device, void* stream);
/* GATConv's attention logits (the reference's gatconv.py:137-138, two torch multiply +
 * sum pairs): el[i, h] = sum_d feat_src[i, h, d] attn_l[h, d] for i < n_src, er[i, h] =
 * sum_d feat_dst[i, h, d] attn_r[h, d] for i < n_dst, in one pass; feat_dst NULL = the same
 * table as feat_src (n_dst == n_src).  Row-major fp32 device pointers, the inputs 16-byte
 * aligned.  The backward writes grad_src = grad_el attn_l (+ grad_er attn_r for one table)
 * and grad_dst = grad_er attn_r (two tables), and per-thread partials of the parameter
 * gradients: DGLMIGatAttnLogitsPartials(...) records of 8 floats, record t = {sum over its
 * rows of grad_el feat_src at slot t mod (H D / 4) (4 floats), the same of grad_er
 * feat_dst (4)}; summing the records of each slot in record order gives grad attn_l and
 * grad attn_r.  el / er are bit-identical to torch's (x * a).sum(-1) on MI355X (its
 * pairwise order).  DGLMIGatAttnLogitsSupported: head_dim in {4, 8, 16, 32, 64}, heads *
 * head_dim / 4 dividing 256 (extension). */
int DGLMIGatAttnLogitsSupported(int64_t num_heads, int64_t head_dim);
int64_t DGLMIGatAttnLogitsPartials(int64_t n_src, int64_t n_dst, int64_t num_heads, int64_t head_dim);
int DGLMIGatAttnLogits(const float* feat_src, const float* feat_dst, int64_t n_src, int64_t n_dst,
                       int64_t num_heads, int64_t head_dim, const float* attn_l, const float* attn_r,
                       float* el, float* er, int device, void* stream);
int DGLMIGatAttnLogitsBackward(const float* feat_src, const float* feat_dst, int64_t n_src,
                               int64_t n_dst, int64_t num_heads, int64_t head_dim,
                               const float* attn_l, const float* attn_r, const float* grad_el,
                               const float* grad_er, float* grad_src, float* grad_dst,
                               float* partials, int device, void* stream);
/* out[i, :] = src[index[i], :] for i < n, rows of row_floats floats; index int32
 * (index_bits 32) or int64 (64), device pointers.  Indices are NOT bound-checked: each
 * must lie in [0, rows of src) (dgl.kernel.gather_rows(check=True) verifies on the host
 * side first).  A per-edge operand put into a walk's
 * position order (the position views' operands, GATConv's dropout scale in position
 * space; extension). */
int DGLMIGatherRows(const float* src, int64_t row_floats, const void* index, int index_bits,
                    int64_t n, float* out, void* stream);
int DGLMIEdgeSoftmaxLeakyForward(const DGLMIGraph* graph, const DGLMIArray* logits,
                                 float negative_slope, DGLMIArray* out, void* stream);
int DGLMIEdgeSoftmaxLeakyBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                                  const DGLMIArray* grad_out, const DGLMIArray* logits,
                                  float negative_slope, DGLMIArray* grad_logits, void* stream);

/* ---- the hack's R-GCN layer kernels and neighbour-access benchmark -------------
 * (_CAPI_DGLRgcnLayer0 / 0Backward / 1 / 1Backward / _CAPI_DGLNbAccess,
 * binary_reduce.cc:398-450; kernels binary_reduce_impl.cu:779-1250).  Same argument
 * lists as the reference's PackedFuncs (plus the stream): like the reference, which
 * reads the relation of every edge from its graph object (GetCsrSortedByEdgeType),
 * the entries read it from the graph, DGLMIGraph.etypes (device int32, one entry per
 * edge id, each in [0, num_rels); required when the graph has edges).
 * norm: one float per edge id ((E) or (E, 1)).
 * Every output is overwritten.  Relation transforms run as one dense product over
 * the node rows and every edge only gathers (the hack multiplies per edge).  The
 * hack's Layer0Backward overwrites repeated (source, relation) pairs
 * (binary_reduce_impl.cu:1004) and its Python wrapper drops Layer1's weight
 * gradient (tensor.py:493); these return the exact sums. */
/* Per-graph state of the R-GCN entries (extension, no reference counterpart; the
 * reference sorts its CSR by edge type once per graph inside the graph object,
 * GetCsrSortedByEdgeType, graph.cc:690-746).  Without it every Layer* call
 * gathers the relation of each edge by edge id, gathers norm by edge id and
 * re-sorts the out-CSR by (source, relation).  DGLMIRgcnPrepare builds, on the
 * device and once, for the graph's relations (graph->etypes) and the edge weights
 * `norm` (one float per edge id; NULL = none cached):
 *   layers bit 0 (Layer0 / Layer0Backward): the in-CSR columns etypes[e] * N_src + u
 *     and the out-CSR regrouped by that key;
 *   layers bit 1 (Layer1 / Layer1Backward): the in-CSR columns u * R + etypes[e]
 *     and the out-CSR regrouped by that key;
 * and norm permuted into each walk's position order, so the gathers stream it;
 *   layers bit 2 (fused Layer1 / Layer1Backward): the in-CSR regrouped by
 *     etypes[e] * N_dst + v (relation-major; the out-CSR regrouped by etypes[e] * N_src + u
 *     is out_typed[0], built for bit 0 or bit 2): the fused kernels aggregate each
 *     relation's rows and multiply by W_t in one pass (64-wide gathered rows, outputs
 *     <= 128 wide); results then match the unfused path to fp32 rounding, not bit for bit.
 * Set DGLMIGraph.rgcn to the state; an entry uses it when graph->rgcn->etypes ==
 * graph->etypes, num_rels and the source count match and the layer's bit is set, and
 * uses the cached norm copies only when norm->data == graph->rgcn->norm -- a caller
 * that changes the VALUES behind those pointers must prepare again, or re-gather the
 * norm copies with DGLMIRgcnRefreshNorm (any other norm is read by edge id).  Results
 * are bit-identical with and without the state.  The memory (about 6 int32/float per
 * edge per layer) is the library's until DGLMIRgcnRelease.  Stream-ordered;
 * DGLMIRgcnRelease synchronises the device. */
typedef struct DGLMIRgcnState {
  const int32_t* etypes;    /* the graph->etypes pointer the state was built from */
  const float* norm;        /* the norm pointer of the cached copies, or NULL */
  int32_t num_rels;
  int32_t layers;
  int64_t num_src;
  int64_t nnz;
  const int32_t* positions; /* 0 .. nnz-1: the edge ids of position-ordered walks */
  const int32_t* in_cols[2];   /* [0]: etypes[e] * num_src + u, [1]: u * num_rels + etypes[e] */
  const float* in_norm;        /* norm[in_csr.data[p]] (NULL when no norm was cached) */
  DGLMICsr out_typed[2];       /* out-CSR regrouped by the key of in_cols[i]; data = edge ids */
  const float* out_norm[2];    /* norm per position of out_typed[i] */
  DGLMICsr in_rel;             /* in-CSR regrouped by etypes[e] * N_dst + v; data = edge ids */
  const float* in_rel_norm;    /* norm per position of in_rel */
  void* owner;                 /* library-private */
} DGLMIRgcnState;
int DGLMIRgcnPrepare(const DGLMIGraph* graph, const DGLMIArray* norm, int32_t num_rels,
                     int32_t layers, DGLMIRgcnState* state, void* stream);
/* Re-gathers a state's cached norm copies from `norm` (one float per edge id of the
 * graph the state was prepared on; the state must have been prepared with a norm) and
 * makes norm->data the cached pointer: a new or rewritten edge-weight tensor costs
 * three E-float gathers instead of a new Prepare (no sorts, no allocation). */
int DGLMIRgcnRefreshNorm(const DGLMIGraph* graph, const DGLMIArray* norm, DGLMIRgcnState* state,
                         void* stream);
int DGLMIRgcnRelease(DGLMIRgcnState* state);

/* _CAPI_DGLRgcnLayer0(G, weight, norm, ret):
 * ret[v, :] = sum_{e=(u->v)} weight[etypes[e], u, :] * norm[e];
 * weight (R, N_src, F), ret (N_dst, F). */
int DGLMIRgcnLayer0(const DGLMIGraph* graph, const DGLMIArray* weight, const DGLMIArray* norm,
                    DGLMIArray* ret, void* stream);
/* _CAPI_DGLRgcnLayer0Backward(G, grad_out, norm, grad_weight):
 * grad_weight[t, u, :] = sum over the edges e of relation t out of u of
 * grad_out[v, :] * norm[e]; grad_weight (R, N_src, F). */
int DGLMIRgcnLayer0Backward(const DGLMIGraph* graph, const DGLMIArray* grad_out,
                            const DGLMIArray* norm, DGLMIArray* grad_weight, void* stream);
/* _CAPI_DGLRgcnLayer1(G, hidden, weight, norm, ret):
 * ret[v, :] = sum_e norm[e] * hidden[u, :] . weight[etypes[e]];
 * hidden (N_src, F_in), weight (R, F_in, F_out), ret (N_dst, F_out). */
int DGLMIRgcnLayer1(const DGLMIGraph* graph, const DGLMIArray* hidden, const DGLMIArray* weight,
                    const DGLMIArray* norm, DGLMIArray* ret, void* stream);
/* Extension (no reference counterpart): DGLMIRgcnLayer1 with RelGraphConv's self-loop
 * and bias, ret[v] = agg[v] + bias + hidden[v] . loop_weight (+ epilogue->addend[v]),
 * in the order of relgraphconv.py:186-190 (python/dgl/nn/pytorch/conv/relgraphconv.py),
 * so the module needs no extra GEMM or passes over the output: on the fused kernels the
 * self-loop is one more MFMA pass over the tile's own rows.  loop_weight (F_in, F_out)
 * or NULL, square graphs only; epilogue->bias has F_out floats, epilogue->addend the
 * shape of ret (not aliasing it); row_mul / row_div must be NULL.  NULL loop_weight and
 * epilogue give DGLMIRgcnLayer1. */
int DGLMIRgcnLayer1Ex(const DGLMIGraph* graph, const DGLMIArray* hidden,
                      const DGLMIArray* weight, const DGLMIArray* norm,
                      const DGLMIArray* loop_weight, const DGLMIEpilogue* epilogue,
                      DGLMIArray* ret, void* stream);
/* _CAPI_DGLRgcnLayer1Backward(G, hidden, weight, norm, grad_out, grad_hidden, grad_weight):
 * grad_hidden[u] = sum_{e out of u} norm[e] * grad_out[v] . weight[t]^T;
 * grad_weight[t] = sum_{e of relation t} norm[e] hidden[u]^T grad_out[v]. */
int DGLMIRgcnLayer1Backward(const DGLMIGraph* graph, const DGLMIArray* hidden,
                            const DGLMIArray* weight, const DGLMIArray* norm,
                            const DGLMIArray* grad_out, DGLMIArray* grad_hidden,
                            DGLMIArray* grad_weight, void* stream);
/* Extension: DGLMIRgcnLayer1Backward of DGLMIRgcnLayer1Ex's self-loop as well:
 * grad_hidden also gets grad_out . loop_weight^T, and grad_loop_weight (F_in, F_out; may
 * be NULL) = hidden^T . grad_out.  grad_hidden may be NULL when the input gradient is
 * not wanted (the fused walk then skips its MFMA passes).  NULL loop_weight gives
 * DGLMIRgcnLayer1Backward. */
int DGLMIRgcnLayer1BackwardEx(const DGLMIGraph* graph, const DGLMIArray* hidden,
                              const DGLMIArray* weight, const DGLMIArray* norm,
                              const DGLMIArray* loop_weight, const DGLMIArray* grad_out,
                              DGLMIArray* grad_hidden, DGLMIArray* grad_weight,
                              DGLMIArray* grad_loop_weight, void* stream);
/* _CAPI_DGLNbAccess: the in-neighbour gather benchmark.  Runs `times` in-neighbour
 * row gathers of feat over the in-CSR (the load-balanced copy_u sum, into scratch;
 * the reference's timed kernels read rows without using them) and writes the mean
 * HIP-event time of the launches after the first `warm_up_times` to *avg_us (the
 * reference logs it).  node_map / deg_inc_node_map feed the reference's disabled
 * sharding modes and are ignored.  Synchronises `stream`. */
int DGLMINbAccess(const DGLMIGraph* graph, const DGLMIArray* feat, const int32_t* node_map,
                  const int32_t* deg_inc_node_map, int32_t times, int32_t warm_up_times,
                  double* avg_us, void* stream);

/* ---- partitioning (metis_partition.cc:19-66 replacement; METIS is absent) --
 * Linear Deterministic Greedy over a symmetrised host CSR (int64): node v goes
 * to the part maximising |N(v) ∩ P| (1 - |P| / C), C = ceil(n / k)(1 + slack). */
int DGLMIPartitionLDG(int64_t num_nodes, const int64_t* indptr, const int64_t* indices,
                      int32_t num_parts, double slack, int64_t* assign);

/* Balanced label propagation on the device (extension replacing METIS k-way,
 * metis_partition.cc:19-66, which metis_partition calls on the symmetrised graph,
 * transform.py:589-630).  The symmetrised adjacency is the union of the graph's
 * in-CSR and out-CSR (square graphs only; in_csr.rows required).  `assign`
 * (device int32, num_nodes) holds the initial parts on entry and the final parts
 * on return; each round every node of one hash half proposes the part most of its
 * neighbours sit in when that beats its own, and proposals into part p are
 * accepted with probability min(1, room_p / proposed_weight_p), room_p =
 * (1 + slack) * total / num_parts - load_p.  node_weight: device int32 per node
 * (NULL = 1).  Deterministic for a given seed.  part_loads (host, num_parts) and
 * cut_edges (host; edges whose endpoints sit in different parts) may be NULL.
 * num_parts <= 64.  Synchronises `stream` before returning. */
int DGLMIPartitionLabelProp(const DGLMIGraph* graph, int32_t num_parts, int32_t rounds,
                            double slack, const int32_t* node_weight, uint64_t seed,
                            int32_t* assign, int64_t* part_loads, int64_t* cut_edges,
                            void* stream);

/* ---- measurement utility (bench.py; no reference counterpart) -------------
 * dst[i] = src[i] for num_floats fp32 values (a multiple of 4, both 16-B aligned)
 * by a float4 streaming copy: the access pattern MI355X_MICROARCH.md quotes the
 * achievable HBM rate on, reported beside the 8 TB/s spec. */
int DGLMIStreamCopy(const float* src, float* dst, int64_t num_floats, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* DGLMI_H_ */
