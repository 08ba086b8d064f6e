// Generic g-SpMM / g-SDDMM kernels for gfx950 (every op x reducer x target,
// with and without broadcasting, forward and backward).
//
// Semantics follow the reference CPU UDFs (cpu/binary_reduce_impl.h:24-109,
// cpu/backward_binary_reduce_impl.h:22-161); the execution model does not.
// The reference scatters every edge into its output row with atomics
// (`omp atomic` / CUDA CAS loops, cuda/atomic.cuh:60-119).  Here a reduction
// is owner-computes: the kernel walks the CSR whose rows are the owners of
// the output (in-CSR for reductions to dst, out-CSR for gradients of src),
// a group of L lanes (L = pow2 >= features, <= 64 = one wavefront) owns a
// row, lanes stride over the row's features (coalesced row gathers) and the
// row's edges are folded in CSR order -- no atomics, deterministic order.
// Per-edge outputs (reducer "none", edge gradients) are one group per edge.
//
// These kernels are the complete, always-correct family; the hot
// reduce-to-node cases go to the load-balanced kernels in kernels_spmm.hip.
#include "internal.h"

namespace dglmi {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int64_t ravel(int64_t tx, const Bcast& b, const int64_t* shape,
                                         const int64_t* stride) {
  int64_t out = 0;
  for (int d = 0; d < b.ndim; ++d) {
    const int64_t idx = (tx / b.out_stride[d]) % b.out_shape[d];
    const int64_t lim = shape[d] - 1;
    out += (idx < lim ? idx : lim) * stride[d];
  }
  return out;
}

template <int OP, bool BC>
__device__ __forceinline__ void operand_ptrs(const EdgeArgs& a, int64_t lid, int64_t rid,
                                             int64_t tx, const float*& l, const float*& r) {
  if constexpr (BC) {
    l = a.lhs.data + lid * a.bc.lhs_len * a.len + ravel(tx, a.bc, a.bc.lhs_shape, a.bc.lhs_stride) * a.len;
    r = a.rhs.data + rid * a.bc.rhs_len * a.len + ravel(tx, a.bc, a.bc.rhs_shape, a.bc.rhs_stride) * a.len;
  } else {
    l = a.lhs.data + (lid * a.D + tx) * a.len;
    if constexpr (OP == OP_USE_LHS) r = l;  // never read
    else r = a.rhs.data + (rid * a.D + tx) * a.len;
  }
}

template <int OP, bool BC>
__device__ __forceinline__ float fwd_value(const EdgeArgs& a, int64_t row, int64_t col,
                                           int64_t eid, int64_t tx) {
  const float* l;
  const float* r;
  operand_ptrs<OP, BC>(a, resolve(a.lhs, row, col, eid), resolve(a.rhs, row, col, eid), tx, l, r);
  return op_apply<OP>(l, r, a.len);
}

// Gradient contribution of one edge to element k of the wanted operand's row
// (backward_binary_reduce_impl.h:39-83: grad_e = grad_out * Reducer'(e, out),
// then times the op derivative).
template <int OP, int RED, bool BC>
__device__ __forceinline__ float bwd_value(const EdgeArgs& a, int64_t row, int64_t col,
                                           int64_t eid, int64_t k) {
  const int64_t tx = k / a.len;
  const int64_t i = k - tx * a.len;
  const float* l;
  const float* r;
  operand_ptrs<OP, BC>(a, resolve(a.lhs, row, col, eid), resolve(a.rhs, row, col, eid), tx, l, r);
  int64_t oid = a.fo_role == ROLE_ROW ? row : (a.fo_role == ROLE_COL ? col : eid);
  if (a.fo_map) oid = a.fo_map[oid];
  const float e = op_apply<OP>(l, r, a.len);
  const float o = a.fwd_out[oid * a.D + tx];
  const float go = a.grad_out[oid * a.D + tx];
  const float ge = go * red_backward<RED>(e, o);
  if constexpr (OP == OP_USE_LHS) {
    return a.want == 0 ? ge : 0.0f;
  } else {
    return a.want == 0 ? ge * op_grad_lhs<OP>(l[i], r[i]) : ge * op_grad_rhs<OP>(l[i], r[i]);
  }
}

template <int OP, int RED, bool BC>
__global__ void __launch_bounds__(kBlock) k_node_fwd(EdgeArgs a, int lane_bits) {
  const int L = 1 << lane_bits;
  const int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  if (row >= a.num_rows) return;
  const int64_t beg = a.indptr[row], end = a.indptr[row + 1];
  const int64_t orow = a.out_map ? a.out_map[row] : row;
  float* o = a.out + orow * a.D;
  for (int64_t tx = lane; tx < a.D; tx += L) {
    float acc = red_identity<RED>();
    for (int64_t j = beg; j < end; ++j)
      acc = red_apply<RED>(acc, fwd_value<OP, BC>(a, row, a.indices[j], a.eids[j], tx));
    o[tx] = acc;
  }
}

template <int OP, bool BC>
__global__ void __launch_bounds__(kBlock) k_edge_fwd(EdgeArgs a, int lane_bits) {
  const int L = 1 << lane_bits;
  const int64_t pos = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  if (pos >= a.nnz) return;
  const int64_t row = a.rows[pos], col = a.indices[pos], eid = a.eids[pos];
  const int64_t orow = a.out_map ? a.out_map[eid] : eid;
  float* o = a.out + orow * a.D;
  for (int64_t tx = lane; tx < a.D; tx += L) o[tx] = fwd_value<OP, BC>(a, row, col, eid, tx);
}

template <int OP, int RED, bool BC>
__global__ void __launch_bounds__(kBlock) k_node_bwd(EdgeArgs a, int lane_bits) {
  const int L = 1 << lane_bits;
  const int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  if (row >= a.num_rows) return;
  const int64_t Dg = a.D * a.len;
  const int32_t* gmap = a.want == 0 ? a.lhs.map : a.rhs.map;
  const int64_t grow = gmap ? gmap[row] : row;
  const int64_t beg = a.indptr[row], end = a.indptr[row + 1];
  float* g = a.out + grow * Dg;
  for (int64_t k = lane; k < Dg; k += L) {
    float acc = 0.0f;
    for (int64_t j = beg; j < end; ++j)
      acc += bwd_value<OP, RED, BC>(a, row, a.indices[j], a.eids[j], k);
    g[k] = acc;
  }
}

template <int OP, int RED, bool BC>
__global__ void __launch_bounds__(kBlock) k_edge_bwd(EdgeArgs a, int lane_bits) {
  const int L = 1 << lane_bits;
  const int64_t pos = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  if (pos >= a.nnz) return;
  const int64_t Dg = a.D * a.len;
  const int64_t row = a.rows[pos], col = a.indices[pos], eid = a.eids[pos];
  const int32_t* gmap = a.want == 0 ? a.lhs.map : a.rhs.map;
  const int64_t grow = gmap ? gmap[eid] : eid;
  float* g = a.out + grow * Dg;
  for (int64_t k = lane; k < Dg; k += L) g[k] = bwd_value<OP, RED, BC>(a, row, col, eid, k);
}

// ---- load-balanced reduce-to-row: fixed chunks of CSR positions -----------
// The row-per-group kernels above serialise a hub row's in-edges on one
// group; on power-law graphs (a 10^5-edge hub next to degree-1 rows) that
// group runs alone for most of the launch.  Here a group of L lanes (features
// strided over lanes, up to kNV per lane) owns K consecutive CSR positions,
// folds each row's run in CSR order, writes rows wholly inside the chunk
// directly, the continuation of a row begun in an earlier chunk to the carry
// workspace, and fills zero-degree rows with the identity; k_lb_fixup folds the
// carries into the row head in chunk order (deterministic).
constexpr int kNV = 4;

template <bool BWD>
__device__ __forceinline__ int64_t lb_out_row(const EdgeArgs& a, int64_t r) {
  const int32_t* m = BWD ? (a.want == 0 ? a.lhs.map : a.rhs.map) : a.out_map;
  return m ? m[r] : r;
}

template <int OP, int RED, bool BC, bool BWD>
__global__ void __launch_bounds__(kBlock) k_lb_reduce(EdgeArgs a, int lane_bits) {
  constexpr int U = 4;
  const int L = 1 << lane_bits;
  const int G = kBlock >> lane_bits;
  const int g = threadIdx.x >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // k_lb_fixup's counters
  const int64_t Do = BWD ? a.D * a.len : a.D;
  const int nv = static_cast<int>((Do + L - 1) / L);
  const float I = BWD ? 0.0f : red_identity<RED>();

  auto fill_row = [&](int64_t r) {
    float* o = a.out + lb_out_row<BWD>(a, r) * Do;
#pragma unroll
    for (int v = 0; v < kNV; ++v) {
      const int64_t k = lane + v * L;
      if (v < nv && k < Do) o[k] = I;
    }
  };
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  float acc[kNV];
#pragma unroll
  for (int v = 0; v < kNV; ++v) acc[v] = I;
  auto flush = [&]() {
    float* o = cont ? a.carry + chunk * Do : a.out + lb_out_row<BWD>(a, cur) * Do;
#pragma unroll
    for (int v = 0; v < kNV; ++v) {
      const int64_t k = lane + v * L;
      if (v < nv && k < Do) o[k] = acc[v];
      acc[v] = I;
    }
  };
  for (int64_t base = p0; base < p1; base += U) {
    int64_t rr[U], cc[U], ee[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = base + u < p1 ? base + u : p1 - 1;
      rr[u] = a.rows[p];
      cc[u] = a.indices[p];
      ee[u] = a.eids[p];
    }
    float val[U][kNV];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int v = 0; v < kNV; ++v) {
        const int64_t k = lane + v * L;
        val[u][v] = 0.0f;
        if (v < nv && k < Do && base + u < p1) {
          if constexpr (BWD) val[u][v] = bwd_value<OP, RED, BC>(a, rr[u], cc[u], ee[u], k);
          else val[u][v] = fwd_value<OP, BC>(a, rr[u], cc[u], ee[u], k);
        }
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u >= p1) break;
      if (rr[u] != cur) {
        flush();
        cur = rr[u];
        cont = false;
      }
#pragma unroll
      for (int v = 0; v < kNV; ++v) acc[v] = BWD ? acc[v] + val[u][v] : red_apply<RED>(acc[v], val[u][v]);
    }
  }
  flush();
  fill_empty_rows(a.indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, L, lane, fill_row);
}

template <int RED, bool BWD>
__global__ void __launch_bounds__(kBlock) k_lb_fixup(EdgeArgs a, int lane_bits) {
  const int L = 1 << lane_bits;
  const int G = kBlock >> lane_bits;
  const int lane = threadIdx.x & (L - 1);
  const int64_t chunk = (int64_t)blockIdx.x * G + (threadIdx.x >> lane_bits);
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (chunk == 0 || p0 >= a.nnz) return;
  const int64_t r = a.rows[p0];
  const int64_t start = a.indptr[r];
  if (start >= p0) return;  // not a continuation
  // segmented for long rows (internal.h, kFixSeg)
  const int64_t first = start / K + 1;
  const int64_t last = (a.indptr[r + 1] - 1) / K;
  const int64_t nseg = a.seg_cnt != nullptr ? (last - first + kFixSeg) / kFixSeg : 1;
  if (nseg == 1 ? chunk != first : (chunk - first) % kFixSeg != 0) return;
  const int64_t Do = BWD ? a.D * a.len : a.D;
  auto red = [&](float acc, float t) { return BWD ? acc + t : red_apply<RED>(acc, t); };
  if (nseg > 1) {
    const int64_t cend = chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last;
    for (int64_t k = lane; k < Do; k += L) {
      float acc = a.carry[chunk * Do + k];
      for (int64_t c = chunk + 1; c <= cend; ++c) acc = red(acc, a.carry[c * Do + k]);
      a.carry[chunk * Do + k] = acc;
    }
    if (!seg_arrive_last(a.seg_cnt + first, nseg, L, lane)) return;
  }
  float* o = a.out + lb_out_row<BWD>(a, r) * Do;
  for (int64_t k = lane; k < Do; k += L) {
    float acc = o[k];
    if (nseg > 1)
      for (int64_t sg = 0; sg < nseg; ++sg) acc = red(acc, a.carry[(first + sg * kFixSeg) * Do + k]);
    else
      for (int64_t c = first; c <= last; ++c) acc = red(acc, a.carry[c * Do + k]);
    o[k] = acc;
  }
}

__global__ void k_fill(float* __restrict__ out, int64_t n, float v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = v;
}
__global__ void k_epilogue(float* __restrict__ out, int64_t rows, int64_t F,
                           const float* __restrict__ row_mul, const float* __restrict__ row_div,
                           const float* __restrict__ bias, const float* __restrict__ addend) {
  const int64_t n = rows * F;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / F;
    float x = out[i];
    if (row_mul) x = x * row_mul[r];
    if (row_div) x = x / row_div[r];
    if (bias) x = x + bias[i - r * F];
    if (addend) x = x + addend[i];
    out[i] = x;
  }
}
__global__ void k_fill_i32(int32_t* __restrict__ out, int64_t n, int32_t v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = v;
}

// Lanes per group as a power of two, at most 64: a group must fit in one
// wavefront, because fill_empty_rows (a wave ballot) and seg_arrive_last (a
// shuffle from lane 0) in k_lb_reduce / k_lb_fixup assume it (internal.h).
constexpr int kMaxLaneBits = 6;
static_assert((1 << kMaxLaneBits) <= 64, "a lane group must fit in one wavefront");
int lane_bits_for(int64_t d) {
  int b = 0;
  while ((1 << b) < d && b < kMaxLaneBits) ++b;
  return b;
}

unsigned grid_for(int64_t items, int lane_bits) {
  const int64_t per_block = kBlock >> lane_bits;
  return static_cast<unsigned>((items + per_block - 1) / per_block);
}

// ---- compile-time dispatch ------------------------------------------------
template <template <int, int, bool> class K, typename... Args>
void dispatch3(int op, int red, bool bc, Args&&... args) {
#define DGLMI_RED(OPV, BCV)                                            \
  switch (red) {                                                       \
    case RED_MAX: K<OPV, RED_MAX, BCV>::run(args...); break;           \
    case RED_MIN: K<OPV, RED_MIN, BCV>::run(args...); break;           \
    case RED_PROD: K<OPV, RED_PROD, BCV>::run(args...); break;         \
    default: K<OPV, RED_SUM, BCV>::run(args...); break;                \
  }
#define DGLMI_OP(BCV)                                                  \
  switch (op) {                                                        \
    case OP_ADD: DGLMI_RED(OP_ADD, BCV) break;                         \
    case OP_SUB: DGLMI_RED(OP_SUB, BCV) break;                         \
    case OP_MUL: DGLMI_RED(OP_MUL, BCV) break;                         \
    case OP_DIV: DGLMI_RED(OP_DIV, BCV) break;                         \
    case OP_DOT: DGLMI_RED(OP_DOT, BCV) break;                         \
    default: DGLMI_RED(OP_USE_LHS, false) break;                       \
  }
  if (bc) {
    DGLMI_OP(true)
  } else {
    DGLMI_OP(false)
  }
#undef DGLMI_OP
#undef DGLMI_RED
}

template <int OP, int RED, bool BC>
struct NodeFwd {
  static void run(const EdgeArgs& a, hipStream_t s) {
    if (a.num_rows == 0) return;
    const int lb = lane_bits_for(a.D);
    hipLaunchKernelGGL((k_node_fwd<OP, RED, BC>), dim3(grid_for(a.num_rows, lb)), dim3(kBlock),
                       0, s, a, lb);
  }
};
template <int OP, int RED, bool BC>
struct EdgeFwd {
  static void run(const EdgeArgs& a, hipStream_t s) {
    if (a.nnz == 0) return;
    const int lb = lane_bits_for(a.D);
    hipLaunchKernelGGL((k_edge_fwd<OP, BC>), dim3(grid_for(a.nnz, lb)), dim3(kBlock), 0, s, a, lb);
  }
};
template <int OP, int RED, bool BC>
struct NodeBwd {
  static void run(const EdgeArgs& a, hipStream_t s) {
    if (a.num_rows == 0) return;
    const int lb = lane_bits_for(a.D * a.len);
    hipLaunchKernelGGL((k_node_bwd<OP, RED, BC>), dim3(grid_for(a.num_rows, lb)), dim3(kBlock),
                       0, s, a, lb);
  }
};
template <int OP, int RED, bool BC>
struct EdgeBwd {
  static void run(const EdgeArgs& a, hipStream_t s) {
    if (a.nnz == 0) return;
    const int lb = lane_bits_for(a.D * a.len);
    hipLaunchKernelGGL((k_edge_bwd<OP, RED, BC>), dim3(grid_for(a.nnz, lb)), dim3(kBlock), 0, s,
                       a, lb);
  }
};

template <int OP, int RED, bool BC>
struct LbFwd {
  static void run(const EdgeArgs& a, int lb, unsigned blocks, hipStream_t s) {
    hipLaunchKernelGGL((k_lb_reduce<OP, RED, BC, false>), dim3(blocks), dim3(kBlock), 0, s, a, lb);
    hipLaunchKernelGGL((k_lb_fixup<RED, false>), dim3(blocks), dim3(kBlock), 0, s, a, lb);
  }
};
template <int OP, int RED, bool BC>
struct LbBwd {
  static void run(const EdgeArgs& a, int lb, unsigned blocks, hipStream_t s) {
    hipLaunchKernelGGL((k_lb_reduce<OP, RED, BC, true>), dim3(blocks), dim3(kBlock), 0, s, a, lb);
    hipLaunchKernelGGL((k_lb_fixup<RED, true>), dim3(blocks), dim3(kBlock), 0, s, a, lb);
  }
};

}  // namespace

bool generic_lb_supported(int64_t out_row_len) { return out_row_len >= 1 && out_row_len <= 64 * kNV; }

void launch_generic_lb(int op, int red, bool bcast, bool bwd, const EdgeArgs& a, hipStream_t s) {
  if (a.nnz == 0) return;
  const int64_t Do = bwd ? a.D * a.len : a.D;
  const int lb = lane_bits_for(Do);
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = grid_for(chunks, lb);
  if (red == RED_NONE) red = RED_SUM;
  if (bwd) dispatch3<LbBwd>(op, red, bcast, a, lb, blocks, s);
  else dispatch3<LbFwd>(op, red, bcast, a, lb, blocks, s);
}

void launch_fill(float* out, int64_t n, float value, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_fill, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, out, n, value);
}
void launch_epilogue(float* out, int64_t rows, int64_t F, const float* row_mul,
                     const float* row_div, const float* bias, const float* addend,
                     hipStream_t s) {
  const int64_t n = rows * F;
  if (n <= 0 || (!row_mul && !row_div && !bias && !addend)) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_epilogue, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, out, rows,
                     F, row_mul, row_div, bias, addend);
}
void launch_fill_i32(int32_t* out, int64_t n, int32_t value, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_fill_i32, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, out, n,
                     value);
}

void launch_generic_forward(int op, int red, bool bcast, const EdgeArgs& a, hipStream_t s) {
  if (a.out_role == ROLE_EDGE) dispatch3<EdgeFwd>(op, RED_SUM, bcast, a, s);
  else dispatch3<NodeFwd>(op, red, bcast, a, s);
}

void launch_generic_backward(int op, int red, bool bcast, const EdgeArgs& a, hipStream_t s) {
  // reducer "none" has the derivative of "sum" (functor.h:63-71)
  if (red == RED_NONE) red = RED_SUM;
  const bool edge_owned = (a.want == 0 ? a.lhs.role : a.rhs.role) == ROLE_EDGE;
  if (edge_owned) dispatch3<EdgeBwd>(op, red, bcast, a, s);
  else dispatch3<NodeBwd>(op, red, bcast, a, s);
}

}  // namespace dglmi
