/*
 * oracle/hack_ref.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the hack's own GPU-only entry points of ydwu4/dgl-hack, the
 * PackedFuncs the upstream DGL 0.4 does not have (`_CAPI_DGLFusedGatKernel`,
 * `_CAPI_DGLKernelBackwardFusedGat`, `_CAPI_DGLKernelRgcnLayer0/1[Backward]`,
 * src/kernel/binary_reduce.cc:380-450).  The reference has no CPU build of these
 * kernels, so this file restates the CUDA kernels' arithmetic, thread by thread, in
 * one sequential order:
 *
 *   hack_sort_rows_by_type    Graph::GetCsrSortedByEdgeType, src/graph/graph.cc:690-746
 *                             (std::sort of each row by type; the restatement is the
 *                             stable order, one of the orders std::sort may produce)
 *   hack_fused_gat            gatExpLeakyReluSumKernel + gatSumProdZipDivKernel,
 *                             src/kernel/cuda/binary_reduce_impl.cu:47-112
 *                             (FusedGatKernelImpl, binary_reduce.cc:380-396)
 *   hack_fused_gat_backward   fusedGatBackwardGradFeatSrc :114-151 and
 *                             fusedGatBackwardGradElEr :171-213, dispatched by
 *                             BackwardFusedGatKernelImpl :1248-1308 on the out-CSR
 *   hack_rgcn_layer0          RgcnLayer0KernelImpl :913-933, RgcnLayer0Impl :943-980
 *   hack_rgcn_layer0_backward RgcnLayer0BackwardKernelImpl :982-1008 (in-CSR sorted by
 *                             type, transpose = true: the out-edges of every source)
 *   hack_rgcn_layer1          RgcnLayer1KernelImpl :1082-1117, RgcnLayer1Impl :1119-1155
 *   hack_rgcn_layer1_backward RgcnLayer1BackwardKernelImpl :1157-1194
 *
 * Every accumulation is fp32 (DType = float) in the order one CUDA thread runs it;
 * where the reference adds per-thread partials with atomicAdd (layer 1, the GAT
 * grad_el / grad_er) the restatement adds them in thread-index order.  The caller
 * zero-initialises the outputs the reference's Python side zero-initialises
 * (python/dgl/backend/pytorch/tensor.py:400-402, 452, 486-487).
 *
 * Two reference defects are selectable, so a test can show where the product differs
 * on purpose:
 *   - the layer-0 backward STORES grad_out[v]·norm into grad_weight[t][u] for each
 *     out-edge (u -> v, type t) in turn (:1004), so repeated (u, t) pairs keep only the
 *     last edge's term; `accumulate` = 1 sums them instead (the exact gradient);
 *   - the GAT exponentials skip the running max (exp overflows for logits > 88); the
 *     restatement keeps that, tests stay in range.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Rows of a CSR with each row's entries ordered by edge type (stable counting sort
 * per row).  `types_of_eid[eid]` is the edge's type in [0, num_types). */
int hack_sort_rows_by_type(int64_t n_rows, const int64_t* indptr, const int64_t* ids,
                           const int64_t* eids, const int64_t* types_of_eid, int64_t num_types,
                           int64_t* out_ids, int64_t* out_eids, int64_t* out_types) {
  int64_t* cnt = (int64_t*)calloc((size_t)num_types + 1, sizeof(int64_t));
  if (!cnt) return -1;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t b = indptr[r], e = indptr[r + 1];
    memset(cnt, 0, sizeof(int64_t) * ((size_t)num_types + 1));
    for (int64_t p = b; p < e; ++p) {
      const int64_t t = types_of_eid[eids[p]];
      if (t < 0 || t >= num_types) { free(cnt); return -2; }
      ++cnt[t + 1];
    }
    for (int64_t t = 0; t < num_types; ++t) cnt[t + 1] += cnt[t];
    for (int64_t p = b; p < e; ++p) {
      const int64_t t = types_of_eid[eids[p]];
      const int64_t q = b + cnt[t]++;
      out_ids[q] = ids[p];
      out_eids[q] = eids[p];
      out_types[q] = t;
    }
  }
  free(cnt);
  return 0;
}

/* gatLeakyReluExp, binary_reduce_impl.cu:47-50 (exp of the leaky ReLU, no max) */
static inline float leaky_exp(float v, float slope) { return v > 0 ? expf(v) : expf(slope * v); }

/* Forward on the in-CSR (rows = destinations, ids = sources, eids = edge ids).
 * feat_src (n_src, H, D), el (n_src, H), er (n_dst, H); writes exp (E, H),
 * sum (n_dst, H), ret (n_dst, H, D). */
void hack_fused_gat(int64_t n_dst, const int64_t* indptr, const int64_t* src, const int64_t* eids,
                    int64_t H, int64_t D, const float* feat_src, const float* el, const float* er,
                    float slope, float* exp_out, float* sum_out, float* ret) {
  const int64_t fx = H * D;
  /* gatExpLeakyReluSumKernel :53-81: thread (v, h) */
  for (int64_t v = 0; v < n_dst; ++v)
    for (int64_t h = 0; h < H; ++h) {
      float s = 0.0f;
      for (int64_t p = indptr[v]; p < indptr[v + 1]; ++p) {
        const float t = leaky_exp(el[src[p] * H + h] + er[v * H + h], slope);
        exp_out[eids[p] * H + h] = t;
        s += t;
      }
      sum_out[v * H + h] = s;
    }
  /* gatSumProdZipDivKernel :84-112: thread (v, h, f) */
  for (int64_t v = 0; v < n_dst; ++v)
    for (int64_t h = 0; h < H; ++h)
      for (int64_t f = 0; f < D; ++f) {
        float s = 0.0f;
        for (int64_t p = indptr[v]; p < indptr[v + 1]; ++p)
          s += exp_out[eids[p] * H + h] / sum_out[v * H + h] * feat_src[src[p] * fx + h * D + f];
        ret[v * fx + h * D + f] = s;
      }
}

/* Backward on the out-CSR (rows = sources, ids = destinations, eids = edge ids), from
 * the forward's exp, sum and ret.  grad_feat_src is stored; grad_el and grad_er are
 * accumulated (the caller zero-fills them, tensor.py:400-402). */
void hack_fused_gat_backward(int64_t n_src, const int64_t* indptr, const int64_t* dst,
                             const int64_t* eids, int64_t H, int64_t D, const float* feat_src,
                             const float* el, const float* er, const float* sum_in,
                             const float* exp_in, const float* ret, const float* grad_out,
                             float slope, float* grad_feat_src, float* grad_el, float* grad_er) {
  const int64_t fx = H * D;
  /* fusedGatBackwardGradFeatSrc :114-151: thread (u, h, f) */
  for (int64_t u = 0; u < n_src; ++u)
    for (int64_t h = 0; h < H; ++h)
      for (int64_t f = 0; f < D; ++f) {
        float s = 0.0f;
        for (int64_t p = indptr[u]; p < indptr[u + 1]; ++p) {
          const int64_t v = dst[p];
          s += exp_in[eids[p] * H + h] / sum_in[v * H + h] * grad_out[v * fx + h * D + f];
        }
        grad_feat_src[u * fx + h * D + f] = s;
      }
  /* fusedGatBackwardGradElEr :171-213: thread (u, h, f); the per-f partials reach
   * grad_el[u][h] and grad_er[v][h] by atomicAdd, added here in f order */
  for (int64_t u = 0; u < n_src; ++u)
    for (int64_t h = 0; h < H; ++h)
      for (int64_t f = 0; f < D; ++f) {
        float s = 0.0f;
        const int64_t fo = u * fx + h * D + f;
        for (int64_t p = indptr[u]; p < indptr[u + 1]; ++p) {
          const int64_t v = dst[p];
          const int64_t dof = v * fx + h * D + f;
          const float grad_exp = grad_out[dof] * (feat_src[fo] - ret[dof]) / sum_in[v * H + h];
          const float pre = el[u * H + h] + er[v * H + h];
          const float t2 = grad_exp * exp_in[eids[p] * H + h] * (pre > 0 ? 1.0f : slope);
          s += t2;
          grad_er[v * H + h] += t2;
        }
        grad_el[u * H + h] += s;
      }
}

/* Layer 0 on the in-CSR sorted by type (rows = destinations): weight (R, n_src, F) is
 * the input layer's per-relation embedding table; ret (n_dst, F) is stored. */
void hack_rgcn_layer0(int64_t n_dst, const int64_t* ranges, const int64_t* src_ids,
                      const int64_t* eids, const int64_t* types, const float* weight,
                      int64_t n_src, int64_t F, const float* norm, float* ret) {
  for (int64_t v = 0; v < n_dst; ++v)
    for (int64_t x = 0; x < F; ++x) {
      float agg = 0.0f;
      for (int64_t p = ranges[v]; p < ranges[v + 1]; ++p)
        agg += weight[types[p] * n_src * F + src_ids[p] * F + x] * norm[eids[p]];
      ret[v * F + x] = agg;
    }
}

/* Layer-0 backward on the out-CSR sorted by type (rows = sources).  The reference
 * stores each edge's term (accumulate = 0, last edge of a (u, t) pair wins); the
 * exact gradient sums them (accumulate = 1).  grad_weight (R, n_src, F) arrives
 * zero-filled (tensor.py:452). */
void hack_rgcn_layer0_backward(int64_t n_src, const int64_t* ranges, const int64_t* dst_ids,
                               const int64_t* eids, const int64_t* types, const float* grad_out,
                               const float* norm, int64_t F, int accumulate, float* grad_weight) {
  for (int64_t u = 0; u < n_src; ++u)
    for (int64_t x = 0; x < F; ++x)
      for (int64_t p = ranges[u]; p < ranges[u + 1]; ++p) {
        const float t = grad_out[dst_ids[p] * F + x] * norm[eids[p]];
        float* g = grad_weight + types[p] * n_src * F + u * F + x;
        *g = accumulate ? *g + t : t;
      }
}

/* Layer 1 on the in-CSR sorted by type: hidden (n_src, Y), weight (R, Y, X);
 * thread (y, x) of row v sums h[u][y]·W[t][y][x]·norm over the row, and the Y partials
 * reach ret[v][x] by atomicAdd (here in y order) onto the zero-filled ret
 * (tensor.py:478). */
void hack_rgcn_layer1(int64_t n_dst, const int64_t* ranges, const int64_t* src_ids,
                      const int64_t* eids, const int64_t* types, const float* hidden,
                      const float* weight, int64_t Y, int64_t X, const float* norm, float* ret) {
  for (int64_t v = 0; v < n_dst; ++v)
    for (int64_t y = 0; y < Y; ++y)
      for (int64_t x = 0; x < X; ++x) {
        float agg = 0.0f;
        for (int64_t p = ranges[v]; p < ranges[v + 1]; ++p)
          agg += hidden[src_ids[p] * Y + y] * weight[types[p] * Y * X + y * X + x] * norm[eids[p]];
        ret[v * X + x] += agg;
      }
}

/* Layer-1 backward on the out-CSR sorted by type (rows = sources): thread (y, x) of
 * row u adds g[v][x]·W[t][y][x]·norm over the row into grad_hidden[u][y] and
 * g[v][x]·h[u][y]·norm into grad_weight[t][y][x] per edge (atomics, here in row, then
 * y, x, then position order); both arrive zero-filled (tensor.py:486-487). */
void hack_rgcn_layer1_backward(int64_t n_src, const int64_t* ranges, const int64_t* dst_ids,
                               const int64_t* eids, const int64_t* types, const float* hidden,
                               const float* weight, int64_t Y, int64_t X, const float* norm,
                               const float* grad_out, float* grad_hidden, float* grad_weight) {
  for (int64_t u = 0; u < n_src; ++u)
    for (int64_t y = 0; y < Y; ++y)
      for (int64_t x = 0; x < X; ++x) {
        const float h = hidden[u * Y + y];
        float agg = 0.0f;
        for (int64_t p = ranges[u]; p < ranges[u + 1]; ++p) {
          const float g = grad_out[dst_ids[p] * X + x];
          const float w = weight[types[p] * Y * X + y * X + x];
          const float n = norm[eids[p]];
          agg += g * w * n;
          grad_weight[types[p] * Y * X + y * X + x] += g * h * n;
        }
        grad_hidden[u * Y + y] += agg;
      }
}
