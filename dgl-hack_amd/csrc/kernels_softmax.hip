// Fused edge softmax for gfx950: softmax of edge logits over the in-edges of
// every destination node, forward and backward, H independent values per edge
// (heads).
//
// Reference: python/dgl/nn/pytorch/softmax.py:15-114 composes five kernels
// and two torch ops per forward (copy_e max, e_sub_v, exp, copy_e sum,
// e_div_v) and four per backward, each one a pass over the edges with a
// random gather by edge id.  Here:
//   forward  = k_sm_rows_v<STATS>  (per destination: running max m and sum of
//              exp(s - m), merged online -- one gather of the logits) + its
//              fixup, then k_sm_edges<NORMALIZE> (a[e] = exp(s[e] - m[v]) / l[v],
//              edge-id order: sequential logits in, sequential a out);
//   backward = k_sm_rows_v<DOTSUM> (S[v] = sum_e a[e] * ga[e]) + fixup, then
//              k_sm_edges<GRAD> (gs[e] = a[e] ga[e] - a[e] S[v], the
//              reference's order of operations, softmax.py:103-112).
// Row work is cut into fixed chunks of CSR positions (one wave per chunk), rows cut by a
// chunk boundary are merged in chunk order by the fixup -- deterministic, no atomics.
// On identity-id walks (position views, destination-sorted graphs) the row-owned walk
// (k_sm_owned + k_sm_hub, below) replaces all three.  Two fused modes serve GATConv's
// composition: SoftmaxArgs.act applies leaky_relu where the logits are read (and its
// derivative where the gradient is written), and SoftmaxArgs.node_l computes each logit
// as el[u] + er[v] where it is read, so the per-edge logits are never stored.
#include "internal.h"

#include <algorithm>
#include <climits>

namespace dglmi {
namespace {

constexpr int kBlock = 256;
enum { SM_STATS = 0, SM_DOTSUM = 1 };
enum { SM_NORMALIZE = 0, SM_GRAD = 1 };

template <int H>
__device__ __forceinline__ void ldrow(const float* __restrict__ p, float (&v)[H]) {
  if constexpr (H % 4 == 0) {
#pragma unroll
    for (int i = 0; i < H / 4; ++i) {
      const float4 t = *reinterpret_cast<const float4*>(p + 4 * i);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else if constexpr (H == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  } else {
#pragma unroll
    for (int i = 0; i < H; ++i) v[i] = p[i];
  }
}
template <int H>
__device__ __forceinline__ void strow(float* __restrict__ p, const float (&v)[H]) {
  if constexpr (H % 4 == 0) {
#pragma unroll
    for (int i = 0; i < H / 4; ++i)
      *reinterpret_cast<float4*>(p + 4 * i) = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  } else if constexpr (H == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
#pragma unroll
    for (int i = 0; i < H; ++i) p[i] = v[i];
  }
}

// the fused leaky_relu (SoftmaxArgs.act): forward on loaded logits, backward on a gradient
template <int N>
__device__ __forceinline__ void act_fwd(const SoftmaxArgs& a, float (&x)[N]) {
  if (a.act) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = x[i] > 0.0f ? x[i] : x[i] * a.act_slope;
  }
}
template <int N>
__device__ __forceinline__ void act_bwd(const SoftmaxArgs& a, const float (&x)[N], float (&g)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) g[i] = x[i] > 0.0f ? g[i] : g[i] * a.act_slope;
}

// (m, l) <- merge of two partial softmax states.  Both maxima -inf: the sums add
// (0 + 0, or NaN when either saw a NaN logit), so a NaN is never dropped.
__device__ __forceinline__ void merge(float& m, float& l, float m2, float l2) {
  const float mn = m > m2 ? m : m2;
  const float ms = mn == -INFINITY ? 0.0f : mn;
  l = l * expf(m - ms) + l2 * expf(m2 - ms);
  m = mn;
}

// merge() with one exponential: the larger maximum's own factor is exp(0) = 1.  The
// same (m, l) for finite values; a NaN or +inf anywhere leaves l NaN (so the row's
// softmax is NaN, as with the reference's exp(score - max)); two empty states
// (m = -inf, l = 0) stay empty, and one -inf state with l NaN (a NaN seen while the
// maximum was -inf) keeps its NaN.
__device__ __forceinline__ void merge1(float& m, float& l, float m2, float l2) {
  const bool ge = m >= m2;
  const float hi = ge ? m : m2, lo = ge ? m2 : m;
  const float lhi = ge ? l : l2, llo = ge ? l2 : l;
  l = lhi + llo * expf(lo - (hi == -INFINITY ? 0.0f : hi));
  m = hi;
}

template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_fixup(SoftmaxArgs a) {
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
  float m[H], l[H];
  auto add = [&](int64_t c) {
    float cm[H], cl[H];
    ldrow<H>(a.carry + c * 2 * H, cm);
    if constexpr (MODE == SM_STATS) {
      ldrow<H>(a.carry + c * 2 * H + H, cl);
#pragma unroll
      for (int h = 0; h < H; ++h) merge(m[h], l[h], cm[h], cl[h]);
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) m[h] += cm[h];
    }
  };
  if (nseg > 1) {
    const int64_t cend = chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last;
    ldrow<H>(a.carry + chunk * 2 * H, m);
    if constexpr (MODE == SM_STATS) ldrow<H>(a.carry + chunk * 2 * H + H, l);
    for (int64_t c = chunk + 1; c <= cend; ++c) add(c);
    strow<H>(a.carry + chunk * 2 * H, m);
    if constexpr (MODE == SM_STATS) strow<H>(a.carry + chunk * 2 * H + H, l);
    if (!seg_arrive_last(a.seg_cnt + first, nseg, 1, 0)) return;
  }
  ldrow<H>(a.stat0 + r * H, m);
  if constexpr (MODE == SM_STATS) ldrow<H>(a.stat1 + r * H, l);
  if (nseg > 1)
    for (int64_t sg = 0; sg < nseg; ++sg) add(first + sg * kFixSeg);
  else
    for (int64_t c = first; c <= last; ++c) add(c);
  strow<H>(a.stat0 + r * H, m);
  if constexpr (MODE == SM_STATS) strow<H>(a.stat1 + r * H, l);
}

// One lane per edge; items in edge-id order (coo_dst) or in-CSR order.  (Two or four
// edges in flight per lane, loads issued before any store, measured no faster: 2.98
// against 2.73 ms at H = 8 on the C3 graph.)
template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_edges(SoftmaxArgs a) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < a.nnz; p += stride) {
    int64_t v, e;
    if (a.coo_dst) {
      e = p;
      v = a.coo_dst[p];
    } else {
      e = a.eids[p];
      v = a.rows[p];
    }
    float s[H], x[H], o[H];
    // node logits: the source of this item (edge-id order: coo_src; CSR order: cols)
    auto node_logits = [&](float (&y)[H]) {
      const int64_t u = a.coo_dst ? a.coo_src[p] : a.cols[p];
      float l[H], r[H];
      ldrow<H>(a.node_l + u * H, l);
      ldrow<H>(a.node_r + v * H, r);
#pragma unroll
      for (int h = 0; h < H; ++h) y[h] = l[h] + r[h];
    };
    if (MODE == SM_NORMALIZE && a.node_l != nullptr) node_logits(s);
    else ldrow<H>(a.s + e * H, s);
    if constexpr (MODE == SM_NORMALIZE) {
      float l[H];
      if (a.stat_pk != nullptr) {  // the row's max and sum side by side: one request
        ldrow<H>(a.stat_pk + v * 2 * H, x);
        ldrow<H>(a.stat_pk + v * 2 * H + H, l);
      } else {
        ldrow<H>(a.stat0 + v * H, x);
        ldrow<H>(a.stat1 + v * H, l);
      }
      act_fwd<H>(a, s);
#pragma unroll
      for (int h = 0; h < H; ++h) o[h] = expf(s[h] - x[h]) / l[h];
    } else {
      float g[H], ax[H];
      ldrow<H>(a.stat0 + v * H, x);
      ldrow<H>(a.ga + e * H, g);
      if (a.act) {
        if (a.node_l != nullptr) node_logits(ax);
        else ldrow<H>(a.act_x + e * H, ax);
      }
#pragma unroll
      for (int h = 0; h < H; ++h) o[h] = s[h] * g[h] - s[h] * x[h];
      if (a.act) act_bwd<H>(a, ax, o);
    }
    strow<H>(a.out + e * H, o);
  }
}

// The forward's row statistics packed side by side for the edge pass in edge-id order:
// pk[r] = (max[r, 0..H), sum[r, 0..H)), so an edge's two gathers are one request.
template <int H>
__global__ void __launch_bounds__(kBlock) k_sm_pack(SoftmaxArgs a) {
  const int64_t n = a.num_rows * H;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / H, h = i % H;
    a.stat_pk[r * 2 * H + h] = a.stat0[i];
    a.stat_pk[r * 2 * H + H + h] = a.stat1[i];
  }
}

// k_sm_edges in edge-id order at H <= 2 (round 6): P = 4 / H consecutive edges per lane,
// so every per-edge stream (logits or softmax output, its gradient, the leaky_relu input,
// the COO) is one 16-B (COO at H = 2: 8-B) load or store per lane instead of P; the
// statistics gathers stay per edge (a few MB of rows: L2).  The same operations in the
// same order as k_sm_edges, so the same bits.  Every stream 16-B aligned (quad_edges_ok).
template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_edges_q(SoftmaxArgs a) {
  constexpr int P = 4 / H;
  const int64_t nq = (a.nnz + P - 1) / P;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  auto ld4 = [](const float* __restrict__ base, int64_t e0, int64_t n, float (&x)[4]) {
    if (e0 + P <= n) {
      const float4 t = *reinterpret_cast<const float4*>(base + e0 * H);
      x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = e0 + i / H < n ? base[e0 * H + i] : 0.0f;
    }
  };
  auto ldP = [](const int32_t* __restrict__ base, int64_t e0, int64_t n, int (&r)[P]) {
    if (e0 + P <= n) {
      if constexpr (P == 4) {
        const int4 t = *reinterpret_cast<const int4*>(base + e0);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
      } else {
        const int2 t = *reinterpret_cast<const int2*>(base + e0);
        r[0] = t.x; r[1] = t.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) r[k] = e0 + k < n ? base[e0 + k] : 0;
    }
  };
  for (int64_t qi = (int64_t)blockIdx.x * kBlock + threadIdx.x; qi < nq; qi += stride) {
    const int64_t e0 = qi * P;
    int v[P];
    ldP(a.coo_dst, e0, a.nnz, v);
    float s[4], o[4];
    auto node_logits = [&](float (&y)[4]) {
      int u[P];
      ldP(a.coo_src, e0, a.nnz, u);
#pragma unroll
      for (int k = 0; k < P; ++k) {
        float l[H], r[H];
        ldrow<H>(a.node_l + (int64_t)u[k] * H, l);
        ldrow<H>(a.node_r + (int64_t)v[k] * H, r);
#pragma unroll
        for (int h = 0; h < H; ++h) y[k * H + h] = l[h] + r[h];
      }
    };
    if (MODE == SM_NORMALIZE && a.node_l != nullptr) node_logits(s);
    else ld4(a.s, e0, a.nnz, s);
    float g[4], ax[4];
    if constexpr (MODE == SM_GRAD) {
      ld4(a.ga, e0, a.nnz, g);
      if (a.act) {
        if (a.node_l != nullptr) node_logits(ax);
        else ld4(a.act_x, e0, a.nnz, ax);
      }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
      float x[H];
      if constexpr (MODE == SM_NORMALIZE) {
        float l[H], y[H];
        if (a.stat_pk != nullptr) {
          ldrow<H>(a.stat_pk + (int64_t)v[k] * 2 * H, x);
          ldrow<H>(a.stat_pk + (int64_t)v[k] * 2 * H + H, l);
        } else {
          ldrow<H>(a.stat0 + (int64_t)v[k] * H, x);
          ldrow<H>(a.stat1 + (int64_t)v[k] * H, l);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) y[h] = s[k * H + h];
        act_fwd<H>(a, y);
#pragma unroll
        for (int h = 0; h < H; ++h) o[k * H + h] = expf(y[h] - x[h]) / l[h];
      } else {
        float y[H], axk[H];
        ldrow<H>(a.stat0 + (int64_t)v[k] * H, x);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const int i = k * H + h;
          y[h] = s[i] * g[i] - s[i] * x[h];
          axk[h] = ax[i];
        }
        if (a.act) act_bwd<H>(a, axk, y);
#pragma unroll
        for (int h = 0; h < H; ++h) o[k * H + h] = y[h];
      }
    }
    if (e0 + P <= a.nnz) {
      *reinterpret_cast<float4*>(a.out + e0 * H) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (e0 + i / H < a.nnz) a.out[e0 * H + i] = o[i];
    }
  }
}

// ---------------------------------------------------------------------------
// Row-owned walk (identity edge ids: a position view, or a graph whose edges came
// sorted by destination).  The logits of a row are contiguous, so one wave can own
// whole rows: it reads them once from HBM, reduces them, and re-reads them from the
// cache it has just filled to write the output -- one HBM read and one write per value
// instead of the row pass + edge pass (two HBM reads, plus rows and edge ids).
//
// Window w = positions [w W, (w + 1) W) (one wave each).  The wave owns every row that
// STARTS in its window (ends at most T = 2W positions later), and of rows longer than T
// ("hub" rows) only the positions inside its window (a "piece").  A piece's partial
// state goes to carry slot (w, 0) when the hub row started in an earlier window and
// (w, 1) when it starts in this one (a row longer than W crosses every boundary it
// meets, so a window meets at most those two); k_sm_hub merges a hub row's pieces in
// window order (deterministic, no atomics) and writes its positions.  Lane (j, q) holds
// V = min(H, 4) consecutive values (heads q V ..) of position b + j; L = 64 / (H / V)
// positions per step.  A step inside the current row needs no row ids and no cross-lane
// work (every lane keeps its own running max / sum); only a step that crosses a row
// boundary reads the row ids and reduces across lanes.
#ifndef DGLMI_SM_WSTEPS
#define DGLMI_SM_WSTEPS 32  // steps per window (probe builds vary it)
#endif
// (An LDS-staged form of this walk -- each wave's chunk of whole rows loaded once into
// 36 KiB of LDS by buffer_load ... lds and both sweeps read from there -- holds one
// block of four waves per CU and measured slower: C3 view H = 8 fwd 3.67 / bwd 4.28 ms
// against 2.17 / 3.61 here; profiles/r05_edge_softmax_variants.json)
template <int H, int MODE>
struct OwnedShape {
  static constexpr int V = H < 4 ? H : 4;  // values per lane
  static constexpr int LP = H / V;         // lanes per position
  static constexpr int L = 64 / LP;        // positions per step
  static constexpr int U = 16 / V;         // steps whose loads are issued together
  static constexpr int64_t W = DGLMI_SM_WSTEPS * L;  // window (positions)
  static constexpr int64_t T = 2 * W;                // longer rows are hub rows
};

// e^x as one v_exp_f32 (relative error ~|x| 2^-24; x = s - max <= 0 here)
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// an agent-coherent load (global_load sc1: past this CU's L1) of a value another lane
// of the same wave stored earlier in this kernel
__device__ __forceinline__ float ld_fresh(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// CHUNK: the statistics sweep of the chunked row pass on an edge-id walk (k_sm_rows):
// values gathered through the walk's edge ids, (max, sum) stored as they are (the edge
// pass divides), and the chunk's first row, when it continues from the previous chunk,
// stored to the chunk's carry for k_sm_fixup.
template <int H, int MODE, bool CHUNK = false>
struct OwnedWalk {
  using S = OwnedShape<H, MODE>;
  static constexpr int V = S::V, LP = S::LP, L = S::L, U = S::U;
  static constexpr float kId = MODE == SM_STATS ? -INFINITY : 0.0f;  // identity of m
  const SoftmaxArgs& a;
  int j, q;  // position in the step, head group
  float m[V], l[V];  // this lane's running state (MODE DOTSUM: m = sum, l unused)
  int carry_row = -1;      // CHUNK: the row continued from the previous chunk
  float* carry = nullptr;  // CHUNK: its partial state (2H floats)

  __device__ __forceinline__ OwnedWalk(const SoftmaxArgs& args, int lane)
      : a(args), j(lane / LP), q(lane % LP) { clear(); }
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int v = 0; v < V; ++v) { m[v] = kId; l[v] = 0.0f; }
  }
  __device__ __forceinline__ int64_t off(int64_t p) const { return p * H + q * V; }
  // where position p's values sit in s / ga (the edge id's row on an edge-id walk)
  __device__ __forceinline__ int64_t voff(int64_t p) const {
    if constexpr (CHUNK) return a.eids[p] * H + q * V;
    else return p * H + q * V;
  }
  // the logits of position p in row `row`: stored (a.s), or from the nodes (a.node_l:
  // lhs + rhs as the u_add_v SDDMM adds them)
  __device__ __forceinline__ void logits(int64_t p, int row, float (&x)[V]) const {
    if (a.node_l != nullptr) {
      float l[V], r[V];
      ldrow<V>(a.node_l + (int64_t)a.cols[p] * H + q * V, l);
      ldrow<V>(a.node_r + (int64_t)row * H + q * V, r);
#pragma unroll
      for (int v = 0; v < V; ++v) x[v] = l[v] + r[v];
    } else {
      ldrow<V>(a.s + voff(p), x);
    }
  }
  // the backward's leaky_relu input at position p (row `row`)
  __device__ __forceinline__ void act_input(int64_t p, int row, float (&x)[V]) const {
    if (a.node_l != nullptr) logits(p, row, x);
    else ldrow<V>(a.act_x + off(p), x);
  }
  // positions b + u L + j < pend, all in row `row`
  template <int N>
  __device__ __forceinline__ void accumulate(int64_t b, int64_t pend, int row) {
    float x[N][V], g[MODE == SM_DOTSUM ? N : 1][V];
#pragma unroll
    for (int u = 0; u < N; ++u) {
      const int64_t p = b + u * L + j;
      if (p < pend) {
        if constexpr (MODE == SM_DOTSUM) {
          ldrow<V>(a.s + voff(p), x[u]);
          ldrow<V>(a.ga + voff(p), g[u]);
        } else {
          logits(p, row, x[u]);
          act_fwd<V>(a, x[u]);
        }
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          x[u][v] = kId;
          if constexpr (MODE == SM_DOTSUM) g[u][v] = 0.0f;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if constexpr (MODE == SM_STATS) {
        // one rescale per batch: mn = max(m, x_u); l = l e^(m - mn) + sum e^(x_u - mn).
        // All -inf so far: nothing added (l stays 0); a +inf or NaN logit makes l NaN.
        float mb = x[0][v];
#pragma unroll
        for (int u = 1; u < N; ++u) mb = fmaxf(mb, x[u][v]);
        // (fmaxf skips NaN: with mn = -inf every term is exp(-inf) = 0 except a NaN's)
        const float mn = fmaxf(m[v], mb);
        const float ms = mn == -INFINITY ? 0.0f : mn;
        float s = l[v] * fexp(m[v] - ms);
#pragma unroll
        for (int u = 0; u < N; ++u) s += fexp(x[u][v] - ms);
        l[v] = s;
        m[v] = mn;
      } else {
#pragma unroll
        for (int u = 0; u < N; ++u) m[v] += x[u][v] * g[u][v];
      }
    }
  }
  // fold one value into a lane state
  __device__ __forceinline__ static void fold(float& m, float& l, float x) {
    if constexpr (MODE == SM_STATS)
      merge1(m, l, x, x == INFINITY ? __builtin_nanf("") : (x == -INFINITY ? 0.0f : 1.0f));
    else
      m += x;
  }
  // every lane of head group q ends with the group's reduction (xor butterfly: both
  // partners compute the same commutative merge)
  __device__ __forceinline__ void reduce() {
#pragma unroll
    for (int d = LP; d < 64; d <<= 1)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float m2 = __shfl_xor(m[v], d);
        if constexpr (MODE == SM_STATS) {
          const float l2 = __shfl_xor(l[v], d);
          merge1(m[v], l[v], m2, l2);
        } else {
          m[v] += m2;
        }
      }
  }
  // a finished row's statistics: forward (max, 1 / sum), backward sum(a ga)
  __device__ __forceinline__ void put(int row, const float (&pm)[V], const float (&pl)[V]) const {
    if constexpr (CHUNK) {
      const bool c = row == carry_row;
      float* s0 = c ? carry + q * V : a.stat0 + (int64_t)row * H + q * V;
      float* s1 = c ? carry + H + q * V : a.stat1 + (int64_t)row * H + q * V;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        s0[v] = pm[v];
        if constexpr (MODE == SM_STATS) s1[v] = pl[v];
      }
    } else {
      float* s0 = a.stat0 + (int64_t)row * H + q * V;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        s0[v] = pm[v];
        if constexpr (MODE == SM_STATS) a.stat1[(int64_t)row * H + q * V + v] = 1.0f / pl[v];
      }
    }
  }
  __device__ __forceinline__ void stats_of(int row, float (&sm)[V], float (&si)[V]) const {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      sm[v] = ld_fresh(a.stat0 + (int64_t)row * H + q * V + v);
      si[v] = MODE == SM_STATS ? ld_fresh(a.stat1 + (int64_t)row * H + q * V + v) : 0.0f;
    }
  }
  // the output of positions b + u L + j < pend with their row's statistics
  template <int N>
  __device__ __forceinline__ void emit(int64_t b, int64_t pend, const float (&sm)[V], const float (&si)[V],
                                       int row) const {
    float x[N][V], g[MODE == SM_DOTSUM ? N : 1][V], ax[MODE == SM_DOTSUM ? N : 1][V];
#pragma unroll
    for (int u = 0; u < N; ++u) {
      const int64_t p = b + u * L + j;
      if (p < pend) {
        if constexpr (MODE == SM_DOTSUM) {
          ldrow<V>(a.s + off(p), x[u]);
          ldrow<V>(a.ga + off(p), g[u]);
          if (a.act) act_input(p, row, ax[u]);
        } else {
          logits(p, row, x[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < N; ++u) {
      const int64_t p = b + u * L + j;
      if (p >= pend) continue;
      float o[V];
      if constexpr (MODE == SM_STATS) act_fwd<V>(a, x[u]);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if constexpr (MODE == SM_STATS) o[v] = fexp(x[u][v] - sm[v]) * si[v];
        else o[v] = x[u][v] * g[u][v] - x[u][v] * sm[v];  // softmax.py:103-112's order
      }
      if constexpr (MODE == SM_DOTSUM) {
        if (a.act) act_bwd<V>(a, ax[u], o);
      }
      strow<V>(a.out + off(p), o);
    }
  }

  // rows [s0, s1) complete: statistics, then outputs
  __device__ void span(int64_t s0, int64_t s1) {
    sweep_stats(s0, s1);
    sweep_out(s0, s1);
  }
  // statistics of the rows of [s0, s1) (rows cut by s0 / s1: their partial states)
  __device__ void sweep_stats(int64_t s0, int64_t s1) {
    const int jl_full = L - 1;
    int cur = a.rows[s0];
    int64_t cur_end = a.indptr[cur + 1];
    bool open = true;
    clear();
    for (int64_t b = s0; b < s1;) {
      if (cur_end - b >= U * L) { accumulate<U>(b, s1, cur); b += U * L; continue; }
      if (cur_end - b >= L) { accumulate<1>(b, s1, cur); b += L; continue; }
      // a step that crosses a row boundary (cur ends at or before b + L)
      const int64_t p = b + j;
      const bool valid = p < s1, in_cur = p < cur_end;
      float x[V], g[V];
#pragma unroll
      for (int v = 0; v < V; ++v) { x[v] = kId; g[v] = 0.0f; }
      const int rr = in_cur ? cur : (valid ? a.rows[p] : INT_MAX);
      if (valid) {
        if constexpr (MODE == SM_DOTSUM) {
          ldrow<V>(a.s + voff(p), x);
          ldrow<V>(a.ga + voff(p), g);
        } else {
          logits(p, rr, x);
          act_fwd<V>(a, x);
        }
      }
      if constexpr (MODE == SM_DOTSUM) {
#pragma unroll
        for (int v = 0; v < V; ++v) x[v] *= g[v];
      }
      if (in_cur) {
#pragma unroll
        for (int v = 0; v < V; ++v) fold(m[v], l[v], x[v]);
      }
      reduce();
      if (j == 0) put(cur, m, l);
      const int jl = s1 - b < L ? static_cast<int>(s1 - b) - 1 : jl_full;  // last valid j
      // cur ends at b + jl + 1 only in the span's last step (in a full step that is a
      // step inside cur): the span is done
      if (cur_end > b + jl) {
        open = false;
        b += L;
        continue;
      }
      const int rl = __shfl(rr, jl * LP + q);
      const bool mine = valid && !in_cur;
      if (__ballot(mine && rr != rl) == 0) {
        // one new row from cur_end on: each lane starts its own state
        clear();
        if (mine) {
#pragma unroll
          for (int v = 0; v < V; ++v) fold(m[v], l[v], x[v]);
        }
      } else {
        // rows that start and end inside the step: segmented inclusive scan over j
        float sm[V], sl[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
          sm[v] = kId;
          sl[v] = 0.0f;
          if (mine) fold(sm[v], sl[v], x[v]);
        }
        const int rs = in_cur ? -1 : rr;
#pragma unroll
        for (int d = 1; d < L; d <<= 1) {
          const int r2 = __shfl_up(rs, d * LP);
#pragma unroll
          for (int v = 0; v < V; ++v) {
            const float m2 = __shfl_up(sm[v], d * LP);
            const float l2 = MODE == SM_STATS ? __shfl_up(sl[v], d * LP) : 0.0f;
            if (j >= d && r2 == rs) {
              if constexpr (MODE == SM_STATS) merge1(sm[v], sl[v], m2, l2);
              else sm[v] += m2;
            }
          }
        }
        const int rn = __shfl_down(rs, LP);
        const bool seg_end = mine && (j == jl || rn != rs);
        if (seg_end && rs != rl) put(rs, sm, sl);
        clear();
        if (j == jl) {
#pragma unroll
          for (int v = 0; v < V; ++v) { m[v] = sm[v]; l[v] = sl[v]; }
        }
      }
      cur = rl;
      cur_end = a.indptr[cur + 1];
      b += L;
    }
    if (open) {
      reduce();
      if (j == 0) put(cur, m, l);
    }
  }
  // the outputs of the complete rows [s0, s1) from their statistics
  __device__ void sweep_out(int64_t s0, int64_t s1) {
    const int jl_full = L - 1;
    // this wave's row statistics, stored by sweep_stats's j == 0 lanes, before any lane
    // reads them back (ld_fresh: L2, the point of coherence)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);  // every store of this wave performed at L2
    __builtin_amdgcn_wave_barrier();
    int cur = a.rows[s0];
    int64_t cur_end = a.indptr[cur + 1];
    float cm[V], ci[V];
    stats_of(cur, cm, ci);
    for (int64_t b = s0; b < s1;) {
      if (cur_end - b >= U * L) { emit<U>(b, s1, cm, ci, cur); b += U * L; continue; }
      if (cur_end - b >= L) { emit<1>(b, s1, cm, ci, cur); b += L; continue; }
      const int64_t p = b + j;
      const bool valid = p < s1, in_cur = p < cur_end;
      const int rr = in_cur ? cur : (valid ? a.rows[p] : cur);
      float rm[V], ri[V];
      if (in_cur) {
#pragma unroll
        for (int v = 0; v < V; ++v) { rm[v] = cm[v]; ri[v] = ci[v]; }
      } else {
        stats_of(rr, rm, ri);
      }
      emit<1>(b, s1, rm, ri, rr);
      const int jl = s1 - b < L ? static_cast<int>(s1 - b) - 1 : jl_full;
      if (cur_end <= b + jl) {
        cur = __shfl(rr, jl * LP + q);
        cur_end = a.indptr[cur + 1];
        stats_of(cur, cm, ci);
      }
      b += L;
    }
  }
  // partial state of hub row positions [pa, pb) -> carry slot
  __device__ void piece(int64_t pa, int64_t pb, float* slot, int row) {
    clear();
    for (int64_t b = pa; b < pb; b += U * L) accumulate<U>(b, pb, row);
    reduce();
    if (j == 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        slot[q * V + v] = m[v];
        if constexpr (MODE == SM_STATS) slot[H + q * V + v] = l[v];
      }
    }
  }
  // the outputs of hub row positions [pa, pb) from the row's statistics
  __device__ void emit_range(int64_t pa, int64_t pb, const float (&sm)[V], const float (&si)[V], int row) const {
    for (int64_t b = pa; b < pb; b += U * L) emit<U>(b, pb, sm, si, row);
  }
  static constexpr int64_t W = S::W, T = S::T;
};

// ---------------------------------------------------------------------------
// The row-owned walk with four values per lane, H <= 4 (round 6).  At H = 1 the walk
// above loads 4 B per lane (one position), and its steps wait on one another: a step's
// loads are issued only after the previous step's row logic, and every row end costs a
// dependent indptr load (profiles/r06_edge_softmax_h1_pmc.json: 79 % of the cycles
// waiting on memory).  Here
// * lane j of a step holds the P = 4 / H positions B + P j .. B + P j + P - 1 with all
//   their heads -- one 16-B load per lane and array, L = 64 P positions a step; every
//   step starts at a multiple of P, so every load is aligned, and positions outside the
//   range being walked are masked (element by element, only in a quad the range cuts);
// * the loads of U steps are issued together whatever the rows do: the row of every
//   position comes from a slice of the row offsets held one per lane (lane t: the start
//   of row rb + t), so a row end needs no memory access -- only batches with more than
//   kEnds row ends (short rows) read the row ids, and the slice is reloaded when the
//   walk leaves it;
// * a step that crosses a row end folds each lane's positions into lane-local segments
//   first: a row that starts and ends inside one lane is finished there, and each lane's
//   first and last segments take part in the segmented scan over the lanes (a lane's
//   first segment continues the previous lane's scan);
// * the statistics of the span's first kRows rows are kept in LDS too, so the output
//   sweep reads them there (no fence and no L2 round trip).
// Windows (2048 positions, as above; 1024 / 4096 measured slower), the hub threshold 2W
// and the two carry slots per window are the walk above's scheme, so k_sm_hub serves
// both.  32-bit row offsets only (the 64-bit layout keeps the walk above).  C3 view, H = 1
// fwd / bwd 0.64 / 0.96 -> 0.36 / 0.44 ms (profiles/r06_edge_softmax_quad_probe.json).
template <int H>
struct QuadShape {
  static_assert(H == 1 || H == 2 || H == 4, "four values per lane: H <= 4");
  static constexpr int P = 4 / H;   // positions per lane
  static constexpr int L = 64 * P;  // positions per step
#ifndef DGLMI_SMQ_U
#define DGLMI_SMQ_U 2
#endif
#ifndef DGLMI_SMQ_U4
#define DGLMI_SMQ_U4 4
#endif
  static constexpr int U = H == 4 ? DGLMI_SMQ_U4 : DGLMI_SMQ_U;  // steps whose loads are issued together
#ifndef DGLMI_SMQ_W
#define DGLMI_SMQ_W 2048
#endif
  static constexpr int64_t W = DGLMI_SMQ_W;  // window (positions)
  static constexpr int64_t T = 2 * W;
  static_assert(W % L == 0, "windows of whole steps");
};

template <int H, int MODE>
struct QuadWalk {
  using S = QuadShape<H>;
  static constexpr int P = S::P, L = S::L, U = S::U;
  static constexpr int V = H, q = 0;  // every lane holds all heads (k_sm_hub's carry offsets)
  static constexpr int W = S::W, T = S::T;
  static constexpr int kRows = 128;  // rows of a span whose statistics stay in LDS
  static constexpr int kEnds = 8;    // row ends per batch taken from the slice
  static constexpr float kId = MODE == SM_STATS ? -INFINITY : 0.0f;  // identity of m
  const SoftmaxArgs& a;
  const int32_t* ip;  // the in-CSR's row offsets
  int j;
  float m[H], l[H];  // this lane's running state (MODE DOTSUM: m = sum, l unused)
  int rb = -(1 << 30), st = 0;  // slice: lane t holds indptr[rb + t] (clamped at the last row)
  float* cache;                 // LDS, kRows x 2H: statistics of rows c0 ..
  int c0 = 0;
  bool spill = false;  // a row past the cache had its statistics stored (read back from L2)

  __device__ __forceinline__ QuadWalk(const SoftmaxArgs& args, int lane, float* lds = nullptr)
      : a(args), ip(static_cast<const int32_t*>(args.indptr.p)), j(lane), cache(lds) { clear(); }
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int h = 0; h < H; ++h) { m[h] = kId; l[h] = 0.0f; }
  }
  __device__ __forceinline__ static int first(int p) { return p - p % P; }
  __device__ __forceinline__ static bool in(int p, int lo, int hi) { return p >= lo && p < hi; }

  // ---- row offsets ----
  __device__ __forceinline__ void slice(int r) {
    rb = r;
    const int t = r + j;
    st = ip[t < a.num_rows ? t : a.num_rows];
  }
  // indptr[r] (r uniform), reloading the slice from r when it does not hold r
  __device__ __forceinline__ int start_of(int r) {
    if (r < rb || r - rb >= 64) slice(r);
    return __shfl(st, r - rb);
  }
  __device__ __forceinline__ int end_of(int r) {
    if (r < rb || r + 1 - rb >= 64) slice(r);
    return __shfl(st, r + 1 - rb);
  }
  // the row holding position p (the slice holds the row's start): the last lane whose
  // start is <= p; a.rows[p] when that is the slice's last lane
  __device__ __forceinline__ int row_holding(int p) {
    const int n = __popcll(__ballot(st <= p));
    return n < 64 ? rb + n - 1 : a.rows[p];
  }
  // the rows of the positions of steps b + u L (u < N), cur's row ends at cur_end: from
  // the slice when it holds the first start past the batch and at most kEnds ends fall
  // inside it, else read (outside [lo, hi) they are not used)
  template <int N>
  __device__ __forceinline__ void batch_rows(int b, int lo, int hi, int cur, int (&rk)[N][P]) {
    const int last = (b + N * L < hi ? b + N * L : hi) - 1;
    if (cur < rb || cur + 1 - rb >= 64) slice(cur);
    const int t0 = cur + 1 - rb;  // lane of cur's end
    const int n = __popcll(__ballot(j >= t0 && st <= last));
#pragma unroll
    for (int u = 0; u < N; ++u)
#pragma unroll
      for (int k = 0; k < P; ++k) rk[u][k] = cur;
    if (n <= kEnds && t0 + n < 64) {
      for (int i = 0; i < n; ++i) {
        const int e = __shfl(st, t0 + i);
#pragma unroll
        for (int u = 0; u < N; ++u)
#pragma unroll
          for (int k = 0; k < P; ++k) rk[u][k] += b + u * L + P * j + k >= e ? 1 : 0;
      }
    } else {
#pragma unroll
      for (int u = 0; u < N; ++u) ldi(a.rows, b + u * L + P * j, lo, hi, rk[u]);
    }
  }

  // a[u] <- a[u + 1]: the next step of a batch moves to slot 0
  template <class Tv, int N, int K>
  __device__ __forceinline__ static void shift(Tv (&v)[N][K]) {
#pragma unroll
    for (int u = 0; u + 1 < N; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k) v[u][k] = v[u + 1][k];
  }

  // ---- quads ----
  // the 4 floats of the quad at q0 (a multiple of P) of an array of H floats per position;
  // positions outside [lo, hi) read as `fill` (and are not loaded)
  __device__ __forceinline__ static void ldq(const float* __restrict__ base, int q0, int lo, int hi,
                                              float (&x)[4], float fill) {
    if (q0 >= lo && q0 + P <= hi) {
      const float4 t = *reinterpret_cast<const float4*>(base + (int64_t)q0 * H);
      x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = in(q0 + i / H, lo, hi) ? base[(int64_t)q0 * H + i] : fill;
    }
  }
  // the P int32 of the quad at q0 (row ids, column ids); -1 outside [lo, hi)
  __device__ __forceinline__ static void ldi(const int32_t* __restrict__ base, int q0, int lo, int hi,
                                              int (&r)[P]) {
    if (q0 >= lo && q0 + P <= hi) {
      if constexpr (P == 4) {
        const int4 t = *reinterpret_cast<const int4*>(base + q0);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
      } else if constexpr (P == 2) {
        const int2 t = *reinterpret_cast<const int2*>(base + q0);
        r[0] = t.x; r[1] = t.y;
      } else {
        r[0] = base[q0];
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) r[k] = in(q0 + k, lo, hi) ? base[q0 + k] : -1;
    }
  }
  // store the quad at q0, only its positions inside [lo, hi)
  __device__ __forceinline__ static void stq(float* __restrict__ base, int q0, int lo, int hi,
                                              const float (&o)[4]) {
    if (q0 >= lo && q0 + P <= hi) {
      *reinterpret_cast<float4*>(base + (int64_t)q0 * H) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (in(q0 + i / H, lo, hi)) base[(int64_t)q0 * H + i] = o[i];
    }
  }
  // the stored logits of the quad (a.s), or lhs + rhs from the nodes (a.node_l: position
  // q0 + k in row rk[k]); kId outside [lo, hi)
  __device__ __forceinline__ void raw(int q0, int lo, int hi, const int (&rk)[P], float (&x)[4]) const {
    if (a.node_l != nullptr) {
      int c[P];
      ldi(a.cols, q0, lo, hi, c);
#pragma unroll
      for (int k = 0; k < P; ++k) {
        float lv[H], rv[H];
        if (in(q0 + k, lo, hi)) {
          ldrow<H>(a.node_l + (int64_t)c[k] * H, lv);
          ldrow<H>(a.node_r + (int64_t)rk[k] * H, rv);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) x[k * H + h] = in(q0 + k, lo, hi) ? lv[h] + rv[h] : kId;
      }
    } else {
      ldq(a.s, q0, lo, hi, x, kId);
    }
  }
  // the forward's values: raw logits with the fused leaky_relu on the positions inside [lo, hi)
  __device__ __forceinline__ void logits(int q0, int lo, int hi, const int (&rk)[P], float (&x)[4]) const {
    raw(q0, lo, hi, rk, x);
    if (a.act) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (in(q0 + i / H, lo, hi)) x[i] = x[i] > 0.0f ? x[i] : x[i] * a.act_slope;
    }
  }
  // the statistics sweep's values of the quad: forward the logits, backward a * ga
  __device__ __forceinline__ void stat_values(int q0, int lo, int hi, const int (&rk)[P],
                                              float (&x)[4]) const {
    if constexpr (MODE == SM_DOTSUM) {
      float g[4];
      ldq(a.s, q0, lo, hi, x, 0.0f);
      ldq(a.ga, q0, lo, hi, g, 0.0f);
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] *= g[i];
    } else {
      logits(q0, lo, hi, rk, x);
    }
  }

  // ---- lane and wave state ----
  // fold one quad's values (kId where masked) into this lane's state: one rescale
  __device__ __forceinline__ void absorb(const float (&x)[4]) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      if constexpr (MODE == SM_STATS) {
        float mb = x[h];
#pragma unroll
        for (int k = 1; k < P; ++k) mb = fmaxf(mb, x[k * H + h]);
        const float mn = fmaxf(m[h], mb);
        const float ms = mn == -INFINITY ? 0.0f : mn;
        float s = l[h] * fexp(m[h] - ms);
#pragma unroll
        for (int k = 0; k < P; ++k) s += fexp(x[k * H + h] - ms);
        l[h] = s;
        m[h] = mn;
      } else {
#pragma unroll
        for (int k = 0; k < P; ++k) m[h] += x[k * H + h];
      }
    }
  }
  __device__ __forceinline__ static void fold(float& m, float& l, float x) {
    OwnedWalk<H, MODE>::fold(m, l, x);
  }
  __device__ __forceinline__ static void merge_into(float& m, float& l, float m2, float l2) {
    if constexpr (MODE == SM_STATS) merge1(m, l, m2, l2);
    else m += m2;
  }
  // every lane ends with the wave's reduction (xor butterfly)
  __device__ __forceinline__ void reduce() {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float m2 = __shfl_xor(m[h], d);
        const float l2 = MODE == SM_STATS ? __shfl_xor(l[h], d) : 0.0f;
        merge_into(m[h], l[h], m2, l2);
      }
  }
  // a finished row's statistics: forward (max, 1 / sum), backward sum(a ga); to the
  // statistics arrays and, for the span's first kRows rows, to the LDS cache
  __device__ __forceinline__ void put(int row, const float (&pm)[H], const float (&pl)[H]) {
    const bool cached = cache != nullptr && row - c0 >= 0 && row - c0 < kRows;
    spill |= !cached;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float i = MODE == SM_STATS ? 1.0f / pl[h] : 0.0f;
      a.stat0[(int64_t)row * H + h] = pm[h];
      if constexpr (MODE == SM_STATS) a.stat1[(int64_t)row * H + h] = i;
      if (cached) {
        cache[(row - c0) * 2 * H + h] = pm[h];
        cache[(row - c0) * 2 * H + H + h] = i;
      }
    }
  }
  __device__ __forceinline__ void stats_of(int row, float (&sm)[H], float (&si)[H]) const {
    if (cache != nullptr && row - c0 >= 0 && row - c0 < kRows) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        sm[h] = cache[(row - c0) * 2 * H + h];
        si[h] = cache[(row - c0) * 2 * H + H + h];
      }
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        sm[h] = ld_fresh(a.stat0 + (int64_t)row * H + h);
        si[h] = MODE == SM_STATS ? ld_fresh(a.stat1 + (int64_t)row * H + h) : 0.0f;
      }
    }
  }
  // the row of the step's position plast, on every lane (jl = its lane, kl = its slot)
  __device__ __forceinline__ static int row_at(const int (&rk)[P], int b, int plast) {
    const int jl = static_cast<int>((plast - b) / P), kl = static_cast<int>((plast - b) % P);
    int r = rk[0];
#pragma unroll
    for (int k = 1; k < P; ++k) r = k == kl ? rk[k] : r;
    return __shfl(r, jl);
  }

  // ---- the statistics sweep ----
  // steps b + u L (u < N) inside row `row` (hub pieces, batches inside one row)
  template <int N>
  __device__ __forceinline__ void accumulate(int b, int lo, int hi, int row) {
    float x[N][4];
    int rk[P];
#pragma unroll
    for (int k = 0; k < P; ++k) rk[k] = row;
#pragma unroll
    for (int u = 0; u < N; ++u) stat_values(b + u * L + P * j, lo, hi, rk, x[u]);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      if constexpr (MODE == SM_STATS) {
        float mb = x[0][h];
#pragma unroll
        for (int u = 0; u < N; ++u)
#pragma unroll
          for (int k = 0; k < P; ++k) mb = fmaxf(mb, x[u][k * H + h]);
        const float mn = fmaxf(m[h], mb);
        const float ms = mn == -INFINITY ? 0.0f : mn;
        float s = l[h] * fexp(m[h] - ms);
#pragma unroll
        for (int u = 0; u < N; ++u)
#pragma unroll
          for (int k = 0; k < P; ++k) s += fexp(x[u][k * H + h] - ms);
        l[h] = s;
        m[h] = mn;
      } else {
#pragma unroll
        for (int u = 0; u < N; ++u)
#pragma unroll
          for (int k = 0; k < P; ++k) m[h] += x[u][k * H + h];
      }
    }
  }
  // a step [bu, bu + L) in which cur ends (at cur_end <= plast, the step's last position
  // in the span); returns the row that continues into the next step
  __device__ __forceinline__ int cross(int bu, int s0, int s1, int plast, const float (&x)[4],
                                       const int (&rk)[P], int cur, int cur_end) {
    const int q0 = bu + P * j;
    // cur's positions (a prefix of the step) into the running state, then cur is done
    float xc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xc[i] = in(q0 + i / H, s0, cur_end) ? x[i] : kId;
    absorb(xc);
    reduce();
    if (j == 0) put(cur, m, l);
    const int rl = row_at(rk, bu, plast);
    // this lane's positions past cur, in lane-local segments: the first (head), the
    // last (tail), and rows that start and end inside the lane (finished here)
    bool has = false, multi = false, other = false;
    int hrow = -1, trow = -1;
    float hm[H], hl[H], tm[H], tl[H];
#pragma unroll
    for (int h = 0; h < H; ++h) { hm[h] = tm[h] = kId; hl[h] = tl[h] = 0.0f; }
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (!in(q0 + k, cur_end, s1)) continue;
      other |= rk[k] != rl;
      if (has && rk[k] != trow) {  // trow's segment ends inside this lane
        if (!multi) {
#pragma unroll
          for (int h = 0; h < H; ++h) { hm[h] = tm[h]; hl[h] = tl[h]; }
          hrow = trow;
          multi = true;
        } else {
          put(trow, tm, tl);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) { tm[h] = kId; tl[h] = 0.0f; }
      }
      has = true;
      trow = rk[k];
#pragma unroll
      for (int h = 0; h < H; ++h) fold(tm[h], tl[h], x[k * H + h]);
    }
    if (!multi) hrow = trow;
    if (__ballot(other) == 0) {
      // one new row (rl) from cur_end on: each lane keeps its own state of it
#pragma unroll
      for (int h = 0; h < H; ++h) { m[h] = tm[h]; l[h] = tl[h]; }
      return rl;
    }
    // segmented inclusive scan of the lanes' last segments over j
    const int rs = trow;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int r2 = __shfl_up(rs, d);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float m2 = __shfl_up(tm[h], d);
        const float l2 = MODE == SM_STATS ? __shfl_up(tl[h], d) : 0.0f;
        if (j >= d && r2 == rs) merge_into(tm[h], tl[h], m2, l2);
      }
    }
    // a lane's first segment continues the previous lane's scan
    const int rp = __shfl_up(rs, 1);
    const int hn = __shfl_down(hrow, 1);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float m2 = __shfl_up(tm[h], 1);
      const float l2 = MODE == SM_STATS ? __shfl_up(tl[h], 1) : 0.0f;
      if (multi && j >= 1 && rp == hrow) merge_into(hm[h], hl[h], m2, l2);
    }
    if (multi) put(hrow, hm, hl);
    if (has && (j == 63 || hn != rs) && rs != rl) put(rs, tm, tl);
    clear();
    if (j == static_cast<int>((plast - bu) / P)) {
#pragma unroll
      for (int h = 0; h < H; ++h) { m[h] = tm[h]; l[h] = tl[h]; }
    }
    return rl;
  }
  // statistics of the complete rows [s0, s1), cur = the row at s0
  __device__ void sweep_stats(int s0, int s1, int cur) {
    int cur_end = end_of(cur);
    clear();
    for (int b = first(s0); b < s1; b += U * L) {
      const int last = (b + U * L < s1 ? b + U * L : s1) - 1;
      if (cur_end > last) {  // the batch inside cur
        accumulate<U>(b, s0, s1, cur);
        continue;
      }
      int rk[U][P];
      batch_rows<U>(b, s0, s1, cur, rk);
      float x[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) stat_values(b + u * L + P * j, s0, s1, rk[u], x[u]);
      // one step at a time (the batch shifts down: one copy of the step logic in the code)
#pragma unroll 1
      for (int u = 0; u < U; ++u) {
        const int bu = b + u * L;
        if (bu >= s1) break;
        const int plast = (bu + L < s1 ? bu + L : s1) - 1;
        if (cur_end > plast) {
          absorb(x[0]);
        } else {
          cur = cross(bu, s0, s1, plast, x[0], rk[0], cur, cur_end);
          cur_end = end_of(cur);
        }
        shift(x);
        shift(rk);
      }
    }
    reduce();
    if (j == 0) put(cur, m, l);
  }

  // ---- the output sweep ----
  // the backward's leaky_relu input of the quad
  __device__ __forceinline__ void act_input(int q0, int lo, int hi, const int (&rk)[P],
                                            float (&x)[4]) const {
    if (a.node_l != nullptr) raw(q0, lo, hi, rk, x);
    else ldq(a.act_x, q0, lo, hi, x, 0.0f);
  }
  // the values the output sweep reads for the quad at q0
  __device__ __forceinline__ void out_values(int q0, int lo, int hi, const int (&rk)[P], float (&x)[4],
                                             float (&g)[4], float (&ax)[4]) const {
    if constexpr (MODE == SM_DOTSUM) {
      ldq(a.s, q0, lo, hi, x, 0.0f);
      ldq(a.ga, q0, lo, hi, g, 0.0f);
      if (a.act) act_input(q0, lo, hi, rk, ax);
    } else {
      logits(q0, lo, hi, rk, x);
    }
  }
  // the output of one quad from its values and its positions' statistics
  __device__ __forceinline__ void out_quad(int q0, int lo, int hi, const float (&x)[4],
                                           const float (&g)[4], const float (&ax)[4], const float (&sm)[P][H],
                                           const float (&si)[P][H]) const {
    float o[4];
#pragma unroll
    for (int k = 0; k < P; ++k)
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int i = k * H + h;
        if constexpr (MODE == SM_STATS) {
          o[i] = fexp(x[i] - sm[k][h]) * si[k][h];
        } else {
          o[i] = x[i] * g[i] - x[i] * sm[k][h];  // softmax.py:103-112's order
          if (a.act) o[i] = ax[i] > 0.0f ? o[i] : o[i] * a.act_slope;
        }
      }
    stq(a.out, q0, lo, hi, o);
  }
  __device__ __forceinline__ static void same_stats(const float (&cm)[H], const float (&ci)[H], float (&sm)[P][H],
                                                    float (&si)[P][H]) {
#pragma unroll
    for (int k = 0; k < P; ++k)
#pragma unroll
      for (int h = 0; h < H; ++h) { sm[k][h] = cm[h]; si[k][h] = ci[h]; }
  }
  // the outputs of steps b + u L (u < N), every position inside [lo, hi) in row `row`
  template <int N>
  __device__ __forceinline__ void emit(int b, int lo, int hi, const float (&cm)[H], const float (&ci)[H],
                                       int row) const {
    float x[N][4], g[N][4], ax[N][4];
    int rk[P];
#pragma unroll
    for (int k = 0; k < P; ++k) rk[k] = row;
#pragma unroll
    for (int u = 0; u < N; ++u) out_values(b + u * L + P * j, lo, hi, rk, x[u], g[u], ax[u]);
    float sm[P][H], si[P][H];
    same_stats(cm, ci, sm, si);
#pragma unroll
    for (int u = 0; u < N; ++u) out_quad(b + u * L + P * j, lo, hi, x[u], g[u], ax[u], sm, si);
  }
  // the outputs of the complete rows [s0, s1) (cur = the row at s0) from their statistics
  __device__ void sweep_out(int s0, int s1, int cur) {
    if (__ballot(spill) != 0) {
      // statistics of rows past the cache are read back from L2: this wave's stores first
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_s_waitcnt(0);
    }
    __builtin_amdgcn_wave_barrier();
    int cur_end = end_of(cur);
    float cm[H], ci[H];
    stats_of(cur, cm, ci);
    for (int b = first(s0); b < s1; b += U * L) {
      const int last = (b + U * L < s1 ? b + U * L : s1) - 1;
      if (cur_end > last) {
        emit<U>(b, s0, s1, cm, ci, cur);
        continue;
      }
      int rk[U][P];
      batch_rows<U>(b, s0, s1, cur, rk);
      float x[U][4], g[U][4], ax[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) out_values(b + u * L + P * j, s0, s1, rk[u], x[u], g[u], ax[u]);
#pragma unroll 1
      for (int u = 0; u < U; ++u) {
        const int bu = b + u * L, q0 = bu + P * j;
        if (bu >= s1) break;
        const int plast = (bu + L < s1 ? bu + L : s1) - 1;
        float sm[P][H], si[P][H];
        same_stats(cm, ci, sm, si);
        if (cur_end <= plast) {
#pragma unroll
          for (int k = 0; k < P; ++k)
            if (in(q0 + k, cur_end, s1)) stats_of(rk[0][k], sm[k], si[k]);
        }
        out_quad(q0, s0, s1, x[0], g[0], ax[0], sm, si);
        if (cur_end <= plast) {
          cur = row_at(rk[0], bu, plast);
          cur_end = end_of(cur);
          stats_of(cur, cm, ci);
        }
        shift(x);
        shift(g);
        shift(ax);
        shift(rk);
      }
    }
  }
  // rows [s0, s1) complete (cur = the row at s0): statistics, then outputs
  __device__ void span(int s0, int s1, int cur) {
    const int rb0 = rb, st0 = st;  // the slice as the span starts (restored for the output sweep)
    c0 = cur;
    sweep_stats(s0, s1, cur);
    rb = rb0;
    st = st0;
    sweep_out(s0, s1, cur);
  }
  // partial state of hub row positions [pa, pb) -> carry slot
  __device__ void piece(int pa, int pb, float* slot, int row) {
    clear();
    for (int b = first(pa); b < pb; b += U * L) accumulate<U>(b, pa, pb, row);
    reduce();
    if (j == 0) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        slot[h] = m[h];
        if constexpr (MODE == SM_STATS) slot[H + h] = l[h];
      }
    }
  }
  __device__ void emit_range(int pa, int pb, const float (&sm)[H], const float (&si)[H], int row) const {
    for (int b = first(pa); b < pb; b += U * L) emit<U>(b, pa, pb, sm, si, row);
  }
};

// The window prologue of the four-values-per-lane walk: the row offsets of the window's
// first 64 rows come in as the walk's slice (one load for both ends of the first row and
// the row the span starts with).
template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_owned_q(SoftmaxArgs a) {
  using Walk = QuadWalk<H, MODE>;
  __shared__ float lds[kBlock / 64][Walk::kRows * 2 * H];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x / 64;
  const int w = (int)blockIdx.x * (kBlock / 64) + wv;
  const int lo = w * Walk::W;
  if (lo >= a.nnz) return;
  const int hi = lo + Walk::W < a.nnz ? lo + Walk::W : a.nnz;
  Walk walk(a, lane, lds[wv]);
  const int r0 = a.rows[lo];
  const int r1 = a.rows[hi - 1];
  walk.slice(r0);
  const int st1 = a.indptr[r1], en1 = a.indptr[r1 + 1];
  const int st0 = walk.start_of(r0), en0 = walk.start_of(r0 + 1);
  int s0 = lo;
  int c = r0;
  if (st0 < lo) {  // a row that started in an earlier window
    if (en0 - st0 > Walk::T) walk.piece(lo, en0 < hi ? en0 : hi, a.carry + (int64_t)(2 * w) * 2 * H, r0);
    s0 = en0;  // a shorter one belongs to the window it started in
    if (s0 >= hi) return;
    c = walk.row_holding(s0);
  }
  int s1 = en1;
  if (en1 - st1 > Walk::T) {  // a hub row starting in this window: its first piece
    walk.piece(st1, hi, a.carry + (int64_t)(2 * w + 1) * 2 * H, r1);
    s1 = st1;
  }
  if (s1 > s0) walk.span(s0, s1, c);
}

template <int H, int MODE, class Walk>
__global__ void __launch_bounds__(kBlock) k_sm_owned(SoftmaxArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t lo = w * Walk::W;
  if (lo >= a.nnz) return;
  const int64_t hi = lo + Walk::W < a.nnz ? lo + Walk::W : a.nnz;
  Walk walk(a, lane);
  const int r0 = a.rows[lo];
  const int64_t st0 = a.indptr[r0], en0 = a.indptr[r0 + 1];
  int64_t s0 = lo;
  if (st0 < lo) {  // a row that started in an earlier window
    if (en0 - st0 > Walk::T) walk.piece(lo, en0 < hi ? en0 : hi, a.carry + (2 * w) * 2 * H, r0);
    s0 = en0;  // a shorter one belongs to the window it started in
  }
  if (s0 >= hi) return;
  const int r1 = a.rows[hi - 1];
  const int64_t st1 = a.indptr[r1], en1 = a.indptr[r1 + 1];
  int64_t s1 = en1;
  if (en1 - st1 > Walk::T) {  // a hub row starting in this window: its first piece
    walk.piece(st1, hi, a.carry + (2 * w + 1) * 2 * H, r1);
    s1 = st1;
  }
  if (s1 > s0) walk.span(s0, s1);
}

// hub rows: merge the row's pieces in window order, then write this window's piece
template <int H, int MODE, class Walk>
__global__ void __launch_bounds__(kBlock) k_sm_hub(SoftmaxArgs a) {
  constexpr int V = Walk::V;
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t lo = w * Walk::W;
  if (lo >= a.nnz) return;
  const int64_t hi = lo + Walk::W < a.nnz ? lo + Walk::W : a.nnz;
  Walk walk(a, lane);
  auto finish = [&](int64_t st, int64_t en, int64_t pa, int64_t pb, int row) {
    const int64_t wf = st / Walk::W, wl = (en - 1) / Walk::W;
    float m[V], l[V];
    const float* c = a.carry + (2 * wf + 1) * 2 * H + walk.q * V;  // the first piece
#pragma unroll
    for (int v = 0; v < V; ++v) {
      m[v] = c[v];
      l[v] = MODE == SM_STATS ? c[H + v] : 0.0f;
    }
    for (int64_t w2 = wf + 1; w2 <= wl; ++w2) {
      const float* c2 = a.carry + (2 * w2) * 2 * H + walk.q * V;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if constexpr (MODE == SM_STATS) merge(m[v], l[v], c2[v], c2[H + v]);
        else m[v] += c2[v];
      }
    }
    if constexpr (MODE == SM_STATS) {
#pragma unroll
      for (int v = 0; v < V; ++v) l[v] = 1.0f / l[v];
      // the hub row's statistics, like every other row's (the window it starts in)
      if (pa == st && walk.j == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          a.stat0[(int64_t)row * H + walk.q * V + v] = m[v];
          a.stat1[(int64_t)row * H + walk.q * V + v] = l[v];
        }
      }
    }
    walk.emit_range(pa, pb, m, l, row);
  };
  const int r0 = a.rows[lo];
  const int64_t st0 = a.indptr[r0], en0 = a.indptr[r0 + 1];
  if (st0 < lo && en0 - st0 > Walk::T) finish(st0, en0, lo, en0 < hi ? en0 : hi, r0);
  const int r1 = a.rows[hi - 1];
  const int64_t st1 = a.indptr[r1], en1 = a.indptr[r1 + 1];
  if (st1 >= lo && en1 - st1 > Walk::T) finish(st1, en1, st1, hi, r1);
}

// The chunked row pass of an edge-id walk (round 5): a wave per chunk of K positions,
// walked like the row-owned walk's statistics sweep -- V heads per lane, every lane
// keeping its own running state inside a row, the cross-lane reduction and the
// segmented scan only on steps that cross a row end -- with the logits gathered through
// the edge ids.  (Round 4's k_sm_rows ran the segmented scan on every step: 1.85e9 VALU
// instructions per C3 H = 8 launch, VALU-bound.)  Outputs as before: the chunk's first
// row, when it continues from the previous chunk, to the chunk's carry; every other row
// to the statistics (max, sum); k_sm_fixup merges in chunk order.
template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_rows_v(SoftmaxArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // k_sm_fixup's counters
  OwnedWalk<H, MODE, true> walk(a, lane);
  const int first_row = a.rows[p0];
  if (p0 > 0 && a.rows[p0 - 1] == first_row) {
    walk.carry_row = first_row;
    walk.carry = a.carry + chunk * 2 * H;
  }
  walk.sweep_stats(p0, p1);
}

template <int H, bool QUAD>
void run_owned(const SoftmaxArgs& a, bool backward, hipStream_t st) {
  auto grid = [&](int64_t W) {
    const int64_t windows = (a.nnz + W - 1) / W;
    return dim3(static_cast<unsigned>((windows + kBlock / 64 - 1) / (kBlock / 64)));
  };
  const dim3 blk(kBlock);
  if constexpr (QUAD) {
    using WS = QuadWalk<H, SM_STATS>;
    using WD = QuadWalk<H, SM_DOTSUM>;
    if (!backward) {
      hipLaunchKernelGGL((k_sm_owned_q<H, SM_STATS>), grid(WS::W), blk, 0, st, a);
      hipLaunchKernelGGL((k_sm_hub<H, SM_STATS, WS>), grid(WS::W), blk, 0, st, a);
    } else {
      hipLaunchKernelGGL((k_sm_owned_q<H, SM_DOTSUM>), grid(WD::W), blk, 0, st, a);
      hipLaunchKernelGGL((k_sm_hub<H, SM_DOTSUM, WD>), grid(WD::W), blk, 0, st, a);
    }
  } else {
    using WS = OwnedWalk<H, SM_STATS>;
    using WD = OwnedWalk<H, SM_DOTSUM>;
    if (!backward) {
      hipLaunchKernelGGL((k_sm_owned<H, SM_STATS, WS>), grid(WS::W), blk, 0, st, a);
      hipLaunchKernelGGL((k_sm_hub<H, SM_STATS, WS>), grid(WS::W), blk, 0, st, a);
    } else {
      hipLaunchKernelGGL((k_sm_owned<H, SM_DOTSUM, WD>), grid(WD::W), blk, 0, st, a);
      hipLaunchKernelGGL((k_sm_hub<H, SM_DOTSUM, WD>), grid(WD::W), blk, 0, st, a);
    }
  }
}

// the four-values-per-lane walk: 32-bit row offsets and positions, and its 16-B loads
// need every per-position array 16-B aligned
bool quad_ok(const SoftmaxArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  return a.quad && !a.indptr.wide && a.nnz < INT_MAX - 8 * 4096 && al(a.rows) && al(a.s) && al(a.out) && (a.ga == nullptr || al(a.ga)) &&
         (a.node_l == nullptr || al(a.cols)) && (!a.act || a.node_l != nullptr || al(a.act_x));
}

// the edge pass in edge-id order with four values per lane: its streams 16-B aligned
bool quad_edges_ok(const SoftmaxArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  return a.quad && a.coo_dst != nullptr && al(a.coo_dst) && al(a.s) && al(a.out) && (a.ga == nullptr || al(a.ga)) &&
         (a.node_l == nullptr || al(a.coo_src)) && (!a.act || a.node_l != nullptr || al(a.act_x));
}

template <int H>
void run(const SoftmaxArgs& a, bool backward, hipStream_t st) {
  if (!a.eids) {
    if constexpr (H <= 4) {
      if (quad_ok(a)) {
        run_owned<H, true>(a, backward, st);
        return;
      }
    }
    run_owned<H, false>(a, backward, st);
    return;
  }
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const dim3 rb(static_cast<unsigned>((chunks + kBlock - 1) / kBlock)), blk(kBlock);
  // k_sm_rows: one wave per chunk
  const dim3 rrb(static_cast<unsigned>((chunks + kBlock / 64 - 1) / (kBlock / 64)));
  const int64_t eb = (a.nnz + kBlock - 1) / kBlock;
  const dim3 ebl(static_cast<unsigned>(eb < 256 * 64 ? eb : 256 * 64));
  bool quad_edges = false;  // the edge-id-order pass with P = 4 / H edges per lane
  if constexpr (H <= 2) quad_edges = quad_edges_ok(a);
  constexpr int64_t PQ = H <= 2 ? 4 / H : 1;  // edges per lane there
  const int64_t qb = (a.nnz + PQ * kBlock - 1) / (PQ * kBlock);
  const dim3 qbl(static_cast<unsigned>(qb < 256 * 64 ? qb : 256 * 64));
  if (!backward) {
    hipLaunchKernelGGL((k_sm_rows_v<H, SM_STATS>), rrb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_STATS>), rb, blk, 0, st, a);
    // edge-id order: the rows' statistics packed for the edge pass (the rows are gathered
    // in random order there; in-CSR order reads them in sequence and keeps the two arrays)
    SoftmaxArgs e = a;
    if (a.coo_dst != nullptr && a.stat_pk != nullptr) {
      const int64_t pb = (a.num_rows * H + kBlock - 1) / kBlock;
      hipLaunchKernelGGL((k_sm_pack<H>), dim3(static_cast<unsigned>(pb < 4096 ? pb : 4096)), blk, 0, st, a);
    } else {
      e.stat_pk = nullptr;
    }
    if (quad_edges) hipLaunchKernelGGL((k_sm_edges_q<H <= 2 ? H : 1, SM_NORMALIZE>), qbl, blk, 0, st, e);
    else hipLaunchKernelGGL((k_sm_edges<H, SM_NORMALIZE>), ebl, blk, 0, st, e);
  } else {
    hipLaunchKernelGGL((k_sm_rows_v<H, SM_DOTSUM>), rrb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_DOTSUM>), rb, blk, 0, st, a);
    if (quad_edges) hipLaunchKernelGGL((k_sm_edges_q<H <= 2 ? H : 1, SM_GRAD>), qbl, blk, 0, st, a);
    else hipLaunchKernelGGL((k_sm_edges<H, SM_GRAD>), ebl, blk, 0, st, a);
  }
}

}  // namespace

bool softmax_supported(int64_t H) { return H == 1 || H == 2 || H == 4 || H == 8 || H == 16; }

// positions per chunk (one wave each): 16 steps of the walk's L positions (64 / (H / V),
// V = min(H, 4) heads per lane), fewer while the graph would give fewer than 2048 waves
int64_t softmax_chunk_edges(int64_t nnz, int64_t H) {
  const int64_t V = H < 4 ? H : 4;
  const int64_t L = H >= 1 && H <= 64 ? 64 / (H / V) : 1;
  int64_t steps = 16;
  while (steps > 1 && nnz / (L * steps) < 2048) steps >>= 1;
  return L * steps;
}

// the row-owned walk's carries: two slots of 2H floats per window
int64_t softmax_owned_carry_bytes(int64_t nnz, int64_t H) {
  int64_t W = 0;  // the smallest window of the walks
  switch (H) {
    case 1: W = std::min({OwnedShape<1, SM_STATS>::W, OwnedShape<1, SM_DOTSUM>::W, QuadShape<1>::W}); break;
    case 2: W = std::min({OwnedShape<2, SM_STATS>::W, OwnedShape<2, SM_DOTSUM>::W, QuadShape<2>::W}); break;
    case 4: W = std::min(OwnedShape<4, SM_STATS>::W, OwnedShape<4, SM_DOTSUM>::W); break;
    case 8: W = std::min(OwnedShape<8, SM_STATS>::W, OwnedShape<8, SM_DOTSUM>::W); break;
    default: W = std::min(OwnedShape<16, SM_STATS>::W, OwnedShape<16, SM_DOTSUM>::W); break;
  }
  return ((nnz + W - 1) / W) * 2 * 2 * H * 4;
}

// the forward's row statistics as (max, sum of exp): the row-owned walk keeps 1 / sum
__global__ void k_sm_invert(float* __restrict__ p, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] = 1.0f / p[i];
}
void launch_sm_row_sums(const SoftmaxArgs& a, hipStream_t s) {
  const int64_t n = a.num_rows * a.H;
  if (a.eids || n <= 0) return;  // the chunked route stores the sum itself
  const int64_t want = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_sm_invert, dim3(static_cast<unsigned>(want < 65536 ? want : 65536)), dim3(kBlock), 0,
                     s, a.stat1, n);
}

void launch_edge_softmax(const SoftmaxArgs& a, bool backward, hipStream_t s) {
  if (a.nnz == 0) return;
  switch (a.H) {
    case 1: run<1>(a, backward, s); break;
    case 2: run<2>(a, backward, s); break;
    case 4: run<4>(a, backward, s); break;
    case 8: run<8>(a, backward, s); break;
    default: run<16>(a, backward, s); break;
  }
}

}  // namespace dglmi
