// Load-balanced g-SpMM (reduce to the row node) for gfx950.
//
// Covers the hot reduce-to-node message functions of GraphConv / GATConv:
//   copy_u  -> v = X[col]              (GCN aggregation, copy_u_sum / copy_u_max)
//   copy_e  -> v = E[eid]              (edge-softmax denominators)
//   u_mul_e -> v = X[col] * E[eid]     (and E broadcast over the head dim, GAT)
// folded with sum / max / min into out[row].
//
// Reference: the same arithmetic as cpu/binary_reduce_impl.h:29-52 with
// ReduceSum/Max/Min (cpu/functor.h:19-48); on GPU the reference calls
// cuSPARSE csrmm2 + a cuBLAS transpose for copy_u_sum
// (cuda/binary_reduce_sum.cu:84-143) and a minigun edge-parallel kernel with
// atomics otherwise (cuda/binary_reduce_impl.cuh:22-54).
//
// Design (MI355X-first):
//  * Work is cut into fixed chunks of K consecutive CSR positions (merge-path
//    style), so a power-law hub with 10^5 in-edges is spread over many chunks
//    while ordinary rows cost one pass: every group does the same work.
//  * A group of L lanes (L * 4 * NV >= F floats) owns a chunk; the chunk's
//    (row, col, eid) triples are staged through LDS B at a time with coalesced
//    loads, then each lane gathers VW-float slices (float4 / float2 / float,
//    the widest dividing F) of U source rows at once
//    (U * 16 B in flight per lane, whole 256-B rows per group at F = 64).
//  * Rows are folded in registers and written once (owner computes, no
//    atomics).  A row cut by a chunk boundary writes its head partial to out
//    and each continuing chunk writes one partial to the carry workspace; a
//    fixup pass folds the carries into out in chunk order, so results are
//    deterministic and independent of scheduling.
//  * Zero-in-degree rows get the reducer identity from a row-parallel share
//    of every group (fill_empty_rows, internal.h): no separate fill pass over
//    `out`, and runs of empty rows are spread over the whole grid.
#include "spmm_chunk.h"

namespace dglmi {
namespace {

// ---------------------------------------------------------------------------
template <int F>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[F]) {
  if constexpr (F % 4 == 0) {
#pragma unroll
    for (int i = 0; i < F / 4; ++i) {
      const float4 t = ld4(p + 4 * i);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else if constexpr (F % 2 == 0) {
#pragma unroll
    for (int i = 0; i < F / 2; ++i) {
      const float2 t = *reinterpret_cast<const float2*>(p + 2 * i);
      v[2 * i] = t.x; v[2 * i + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] = p[i];
  }
}

template <int F>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[F]) {
  if constexpr (F % 4 == 0) {
#pragma unroll
    for (int i = 0; i < F / 4; ++i) st4(p + 4 * i, make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]));
  } else {
#pragma unroll
    for (int i = 0; i < F; ++i) p[i] = v[i];
  }
}

// `hidx` (bcast kind): edge value index of each of the F floats, i / head_dim, and
// `wn` = F / head_dim values per edge, computed once per thread by the caller.
template <int KIND, int F>
__device__ __forceinline__ void lane_value(const FastArgs& a, int32_t col, int64_t eid, float (&v)[F],
                                           const int (&hidx)[F], int wn, int32_t row) {
  if constexpr (KIND == FAST_COL_TIE) {
    float o[F], xr[F];
    load_row<F>(a.x + static_cast<int64_t>(col) * F, v);
    load_row<F>(a.w + static_cast<int64_t>(col) * F, o);
    load_row<F>(a.xr + static_cast<int64_t>(row) * F, xr);
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] = xr[i] == o[i] ? v[i] : 0.0f;
  } else if constexpr (KIND == FAST_COPY_COL) {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    load_row<F>(a.x + c * F, v);
  } else if constexpr (KIND == FAST_COPY_EDGE) {
    const int64_t e = a.x_map ? a.x_map[eid] : eid;
    load_row<F>(a.x + e * F, v);
  } else if constexpr (KIND == FAST_COL_MUL_EDGE) {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    const int64_t e = a.w_map ? a.w_map[eid] : eid;
    float w[F];
    load_row<F>(a.x + c * F, v);
    load_row<F>(a.w + e * F, w);
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] *= w[i];
  } else {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    const int64_t e = a.w_map ? a.w_map[eid] : eid;
    load_row<F>(a.x + c * F, v);
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] *= a.w[e * wn + hidx[i]];
  }
}

template <bool EPI, int F>
__device__ __forceinline__ void epi_row(const FastArgs& a, int64_t r, float (&v)[F]) {
  if constexpr (EPI) {
    const float m = a.row_mul ? a.row_mul[r] : 1.0f;
    const float d = a.row_div ? a.row_div[r] : 1.0f;
#pragma unroll
    for (int i = 0; i < F; ++i) {
      float x = v[i];
      if (a.row_mul) x = x * m;
      if (a.row_div) x = x / d;
      if (a.bias) x = x + a.bias[i];
      if (a.addend) x = x + a.addend[r * F + i];
      v[i] = x;
    }
  }
}

template <int KIND, int RED, int F, bool EPI = false>
__global__ void __launch_bounds__(kBlock) k_lane_reduce(FastArgs a) {
  constexpr int U = 8;
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr) a.seg_cnt[chunk] = 0;  // k_lane_fixup's counters
  const float I = red_identity<RED>();
  float ident[F];
#pragma unroll
  for (int i = 0; i < F; ++i) ident[i] = I;
  int hidx[F];
  const int hd = KIND == FAST_COL_MUL_EDGE_BCAST ? static_cast<int>(a.head_dim) : 1;
#pragma unroll
  for (int i = 0; i < F; ++i) hidx[i] = i / hd;
  const int wn = F / hd;
  auto put_gap = [&](int64_t r) {
    float t[F];
#pragma unroll
    for (int i = 0; i < F; ++i) t[i] = ident[i];
    epi_row<EPI, F>(a, r, t);
    store_row<F>(a.out + r * F, t);
  };
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  float acc[F];
#pragma unroll
  for (int i = 0; i < F; ++i) acc[i] = I;
  for (int64_t base = p0; base < p1; base += U) {
    int32_t r[U], c[U];
    int64_t e[U];
    if (base + U <= p1) {
      const int4 r0 = *reinterpret_cast<const int4*>(a.rows + base);
      const int4 r1 = *reinterpret_cast<const int4*>(a.rows + base + 4);
      const int4 c0 = *reinterpret_cast<const int4*>(a.indices + base);
      const int4 c1 = *reinterpret_cast<const int4*>(a.indices + base + 4);
      r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w; r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
      c[0] = c0.x; c[1] = c0.y; c[2] = c0.z; c[3] = c0.w; c[4] = c1.x; c[5] = c1.y; c[6] = c1.z; c[7] = c1.w;
      if constexpr (needs_eid<KIND>()) {
        if (!a.eids) {  // identity edge ids (a position view's walk)
#pragma unroll
          for (int u = 0; u < U; ++u) e[u] = base + u;
        } else if (a.eids.wide) {
#pragma unroll
          for (int u = 0; u < U; ++u) e[u] = a.eids[base + u];
        } else {
          const int32_t* ep = static_cast<const int32_t*>(a.eids.p) + base;
          const int4 e0 = *reinterpret_cast<const int4*>(ep);
          const int4 e1 = *reinterpret_cast<const int4*>(ep + 4);
          e[0] = e0.x; e[1] = e0.y; e[2] = e0.z; e[3] = e0.w; e[4] = e1.x; e[5] = e1.y; e[6] = e1.z; e[7] = e1.w;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = base + u < p1;
        r[u] = ok ? a.rows[base + u] : INT_MAX;
        c[u] = ok ? a.indices[base + u] : 0;
        if constexpr (needs_eid<KIND>()) e[u] = ok ? (a.eids ? a.eids[base + u] : base + u) : 0;
      }
    }
    float v[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r[u] != INT_MAX) lane_value<KIND, F>(a, c[u], needs_eid<KIND>() ? e[u] : 0, v[u], hidx, wn, r[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r[u] == INT_MAX) break;
      if (r[u] != cur) {
        if (!cont) epi_row<EPI, F>(a, cur, acc);
        store_row<F>(cont ? a.carry + chunk * F : a.out + cur * F, acc);
#pragma unroll
        for (int i = 0; i < F; ++i) acc[i] = I;
        cur = r[u];
        cont = false;
      }
#pragma unroll
      for (int i = 0; i < F; ++i) acc[i] = red_apply<RED>(acc[i], v[u][i]);
    }
  }
  if (!cont && !(EPI && p1 < a.nnz && a.rows[p1] == cur)) epi_row<EPI, F>(a, cur, acc);
  store_row<F>(cont ? a.carry + chunk * F : a.out + cur * F, acc);
  fill_empty_rows(a.indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, 1, 0, put_gap);
}

template <int RED, int F, bool EPI = false>
__global__ void __launch_bounds__(kBlock) k_lane_fixup(FastArgs a) {
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (chunk == 0 || p0 >= a.nnz) return;
  const int64_t r = a.rows[p0];
  const int64_t start = a.indptr[r];
  if (start >= p0) return;  // not a continuation
  // segmented for long rows (internal.h, kFixSeg); one lane per chunk
  const int64_t first = start / K + 1;
  const int64_t last = (a.indptr[r + 1] - 1) / K;
  const int64_t nseg = a.seg_cnt != nullptr ? (last - first + kFixSeg) / kFixSeg : 1;
  if (nseg == 1 ? chunk != first : (chunk - first) % kFixSeg != 0) return;
  float acc[F];
  auto add = [&](int64_t c) {
    float t[F];
    load_row<F>(a.carry + c * F, t);
#pragma unroll
    for (int i = 0; i < F; ++i) acc[i] = red_apply<RED>(acc[i], t[i]);
  };
  if (nseg > 1) {
    const int64_t cend = chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last;
    load_row<F>(a.carry + chunk * F, acc);
    for (int64_t c = chunk + 1; c <= cend; ++c) add(c);
    store_row<F>(a.carry + chunk * F, acc);
    if (!seg_arrive_last(a.seg_cnt + first, nseg, 1, 0)) return;
  }
  load_row<F>(a.out + r * F, acc);
  if (nseg > 1)
    for (int64_t sg = 0; sg < nseg; ++sg) add(first + sg * kFixSeg);
  else
    for (int64_t c = first; c <= last; ++c) add(c);
  epi_row<EPI, F>(a, r, acc);
  store_row<F>(a.out + r * F, acc);
}


template <int KIND, int RED, int F>
void run_lane(const FastArgs& a, hipStream_t s) {
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = static_cast<unsigned>((chunks + kBlock - 1) / kBlock);
  if constexpr (RED == RED_SUM) {
    if (has_epi(a)) {
      hipLaunchKernelGGL((k_lane_reduce<KIND, RED, F, true>), dim3(blocks), dim3(kBlock), 0, s, a);
      if (chunks > 1)
        hipLaunchKernelGGL((k_lane_fixup<RED, F, true>), dim3(blocks), dim3(kBlock), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((k_lane_reduce<KIND, RED, F>), dim3(blocks), dim3(kBlock), 0, s, a);
  if (chunks > 1) hipLaunchKernelGGL((k_lane_fixup<RED, F>), dim3(blocks), dim3(kBlock), 0, s, a);
}

template <int KIND, int RED>
void run_lane_f(const FastArgs& a, hipStream_t s) {
  switch (a.F) {
    case 1: run_lane<KIND, RED, 1>(a, s); break;
    case 2: run_lane<KIND, RED, 2>(a, s); break;
    case 3: run_lane<KIND, RED, 3>(a, s); break;
    case 4: run_lane<KIND, RED, 4>(a, s); break;
    case 5: run_lane<KIND, RED, 5>(a, s); break;
    case 6: run_lane<KIND, RED, 6>(a, s); break;
    case 7: run_lane<KIND, RED, 7>(a, s); break;
    case 8: run_lane<KIND, RED, 8>(a, s); break;
    case 12: run_lane<KIND, RED, 12>(a, s); break;
    default: break;
  }
}


template <int KIND, int RED>
void run_cfg(const FastArgs& a, IdxPtr indptr, hipStream_t s) {
  // FAST_COL_MUL_POS has its own kernel only for float4 rows; elsewhere it is the
  // broadcast kind with identity edge ids (the same values, the per-lane weight load)
  constexpr int K2 = KIND == FAST_COL_MUL_POS ? FAST_COL_MUL_EDGE_BCAST : KIND;
  if (a.F < 16 && lane_kernel_width(a.F)) {
    run_lane_f<K2, RED>(a, s);
    return;
  }
  switch (fast_vw(a.F, K2, a.head_dim)) {
    case 4: run_vw<KIND, RED, 4>(a, indptr, s); break;
    case 2: launch_fast_chunk_vw2(K2, RED, a, s); break;
    default: launch_fast_chunk_vw1(K2, RED, a, s); break;
  }
}

__global__ void k_mark_cold(const int32_t* __restrict__ cols, int64_t nnz, IdxPtr deg_indptr,
                            int32_t thresh, int32_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < nnz; p += stride) {
    const int32_t c = cols[p];
    const int64_t d = deg_indptr[c + 1] - deg_indptr[c];
    out[p] = d < thresh ? static_cast<int32_t>(static_cast<uint32_t>(c) | 0x80000000u) : c;
  }
}

}  // namespace

void launch_mark_cold(const int32_t* cols, int64_t nnz, IdxPtr deg_indptr, int32_t thresh,
                      int32_t* out_cols, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t want = (nnz + kBlock - 1) / kBlock;
  const unsigned blocks = static_cast<unsigned>(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(k_mark_cold, dim3(blocks), dim3(kBlock), 0, s, cols, nnz, deg_indptr, thresh,
                     out_cols);
}

int64_t fast_chunk_edges(int64_t nnz, int64_t F) {
  // Enough chunks to give every CU several groups; long chunks otherwise so
  // that fewer rows are cut (each cut row costs one carry write + read).
#if DGLMI_PROBES
  // DGLMI_CHUNK_EDGES overrides (tuning experiments; power of two >= 4).
  if (const char* env = std::getenv("DGLMI_CHUNK_EDGES")) {
    const long v = std::atol(env);
    if (v >= 4 && (v & (v - 1)) == 0) return v;
  }
#endif
  // Measured on M1 (F = 16..256): 512 is best or within 1% (scripts/tune_spmm.py).
  // Narrow rows (F < 16) use one lane per chunk: shorter chunks, more lanes.
  // Small graphs go down to 8 edges per chunk: a launch-bound Cora-size copy_u
  // sum is a chain of dependent loads per chunk, k_chunk_reduce 13.9 us at 32,
  // 8.5 at 16, 7.1 at 8, 6.1 at 4 (scripts/overhead_probe.py under rocprofv3).
  int64_t k = F < 16 ? 128 : 512;
  const int64_t groups_wanted = F < 16 ? 256 /*CUs*/ * 64 * 16 : 256 * 64;
  while (k > 8 && nnz / k < groups_wanted) k >>= 1;
  (void)F;
  return k;
}

int64_t fast_carry_bytes(int64_t nnz, int64_t F) {
  if (nnz == 0) return 0;
  const int64_t k = fast_chunk_edges(nnz, F);
  return (((nnz + k - 1) / k) * F * static_cast<int64_t>(sizeof(float)) + 15) & ~int64_t(15);
}

// carries + one segmented-fixup counter per chunk
int64_t fast_workspace_bytes(int64_t nnz, int64_t F) {
  if (nnz == 0) return 0;
  const int64_t k = fast_chunk_edges(nnz, F);
  return fast_carry_bytes(nnz, F) + ((nnz + k - 1) / k) * static_cast<int64_t>(sizeof(int32_t));
}

bool fast_supported(int kind, int64_t F, int64_t head_dim) {
  if (F < 1) return false;
  if (kind == FAST_COL_MUL_EDGE_BCAST && (head_dim < 1 || F % head_dim != 0)) return false;
  if (F < 16 && lane_kernel_width(F)) return true;
  // 64 lanes x up to 8 float4 or 16 float2 / float slots per lane
  const int vw = fast_vw(F, kind, head_dim);
  return F <= (vw == 1 ? 1024 : 2048);
}

void launch_fast_reduce(int kind, int red, const FastArgs& a, hipStream_t s) {
  const IdxPtr indptr = a.indptr;
  switch (kind) {
    case FAST_COPY_COL:
      if (red == RED_MAX) run_cfg<FAST_COPY_COL, RED_MAX>(a, indptr, s);
      else if (red == RED_MIN) run_cfg<FAST_COPY_COL, RED_MIN>(a, indptr, s);
      else run_cfg<FAST_COPY_COL, RED_SUM>(a, indptr, s);
      break;
    case FAST_COPY_EDGE:
      if (red == RED_MAX) run_cfg<FAST_COPY_EDGE, RED_MAX>(a, indptr, s);
      else if (red == RED_MIN) run_cfg<FAST_COPY_EDGE, RED_MIN>(a, indptr, s);
      else run_cfg<FAST_COPY_EDGE, RED_SUM>(a, indptr, s);
      break;
    case FAST_COL_MUL_EDGE: run_cfg<FAST_COL_MUL_EDGE, RED_SUM>(a, indptr, s); break;
    case FAST_COL_TIE: run_cfg<FAST_COL_TIE, RED_SUM>(a, indptr, s); break;
    case FAST_COL_MUL_POS: run_cfg<FAST_COL_MUL_POS, RED_SUM>(a, indptr, s); break;
    default: run_cfg<FAST_COL_MUL_EDGE_BCAST, RED_SUM>(a, indptr, s); break;
  }
}

}  // namespace dglmi