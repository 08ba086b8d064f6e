// Fused edge softmax for gfx950: softmax of edge logits over the in-edges of
// every destination node, forward and backward, H independent values per edge
// (heads).
//
// Reference: python/dgl/nn/pytorch/softmax.py:15-114 composes five kernels
// and two torch ops per forward (copy_e max, e_sub_v, exp, copy_e sum,
// e_div_v) and four per backward, each one a pass over the edges with a
// random gather by edge id.  Here:
//   forward  = k_sm_rows<STATS>  (per destination: running max m and sum of
//              exp(s - m), merged online -- one gather of the logits) + its
//              fixup, then k_sm_edges<NORMALIZE> (a[e] = exp(s[e] - m[v]) / l[v],
//              edge-id order: sequential logits in, sequential a out);
//   backward = k_sm_rows<DOTSUM> (S[v] = sum_e a[e] * ga[e]) + fixup, then
//              k_sm_edges<GRAD> (gs[e] = a[e] ga[e] - a[e] S[v], the
//              reference's order of operations, softmax.py:103-112).
// Row work is cut into fixed chunks of CSR positions (one lane per chunk,
// whole H-row in registers), rows cut by a chunk boundary are merged in chunk
// order by the fixup -- deterministic, no atomics.
#include "internal.h"

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

// (m, l) <- merge of two partial softmax states
__device__ __forceinline__ void merge(float& m, float& l, float m2, float l2) {
  const float mn = m > m2 ? m : m2;
  if (mn == -INFINITY) return;  // both empty / all -inf
  l = l * expf(m - mn) + l2 * expf(m2 - mn);
  m = mn;
}

template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_rows(SoftmaxArgs a) {
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr) a.seg_cnt[chunk] = 0;  // k_sm_fixup's counters
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  float m[H], l[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = MODE == SM_STATS ? -INFINITY : 0.0f;
    l[h] = 0.0f;
  }
  auto flush = [&]() {
    float* pm = cont ? a.carry + chunk * 2 * H : a.stat0 + cur * H;
    strow<H>(pm, m);
    if constexpr (MODE == SM_STATS) strow<H>(cont ? pm + H : a.stat1 + cur * H, l);
  };
  constexpr int U = 4;
  for (int64_t base = p0; base < p1; base += U) {
    int64_t rr[U];
    float s[U][H], g[U][H];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = base + u < p1 ? base + u : p1 - 1;
      rr[u] = a.rows[p];
      const int64_t e = a.eids[p];
      ldrow<H>(a.s + e * H, s[u]);
      if constexpr (MODE == SM_DOTSUM) ldrow<H>(a.ga + e * H, g[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u >= p1) break;
      if (rr[u] != cur) {
        flush();
#pragma unroll
        for (int h = 0; h < H; ++h) {
          m[h] = MODE == SM_STATS ? -INFINITY : 0.0f;
          l[h] = 0.0f;
        }
        cur = rr[u];
        cont = false;
      }
#pragma unroll
      for (int h = 0; h < H; ++h) {
        if constexpr (MODE == SM_STATS) {
          const float x = s[u][h];
          if (x > m[h]) {
            // the new maximum's own term exp(x - x): 1, or NaN for x = +inf as in
            // the reference's exp(score - max) (softmax.py:70-72)
            l[h] = l[h] * expf(m[h] - x) + (x == INFINITY ? __builtin_nanf("") : 1.0f);
            m[h] = x;
          } else if (x != -INFINITY) {  // a masked logit adds exp(-inf) = 0
            l[h] += expf(x - m[h]);
          }
        } else {
          m[h] += s[u][h] * g[u][h];
        }
      }
    }
  }
  flush();
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

// One lane per edge; items in edge-id order (coo_dst) or in-CSR order.
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
    ldrow<H>(a.s + e * H, s);
    ldrow<H>(a.stat0 + v * H, x);
    if constexpr (MODE == SM_NORMALIZE) {
      float l[H];
      ldrow<H>(a.stat1 + v * H, l);
#pragma unroll
      for (int h = 0; h < H; ++h) o[h] = expf(s[h] - x[h]) / l[h];
    } else {
      float g[H];
      ldrow<H>(a.ga + e * H, g);
#pragma unroll
      for (int h = 0; h < H; ++h) o[h] = s[h] * g[h] - s[h] * x[h];
    }
    strow<H>(a.out + e * H, o);
  }
}

template <int H>
void run(const SoftmaxArgs& a, bool backward, hipStream_t st) {
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const dim3 rb(static_cast<unsigned>((chunks + kBlock - 1) / kBlock)), blk(kBlock);
  const int64_t eb = (a.nnz + kBlock - 1) / kBlock;
  const dim3 ebl(static_cast<unsigned>(eb < 256 * 64 ? eb : 256 * 64));
  if (!backward) {
    hipLaunchKernelGGL((k_sm_rows<H, SM_STATS>), rb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_STATS>), rb, blk, 0, st, a);
    hipLaunchKernelGGL((k_sm_edges<H, SM_NORMALIZE>), ebl, blk, 0, st, a);
  } else {
    hipLaunchKernelGGL((k_sm_rows<H, SM_DOTSUM>), rb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_DOTSUM>), rb, blk, 0, st, a);
    hipLaunchKernelGGL((k_sm_edges<H, SM_GRAD>), ebl, blk, 0, st, a);
  }
}

}  // namespace

bool softmax_supported(int64_t H) { return H == 1 || H == 2 || H == 4 || H == 8 || H == 16; }

int64_t softmax_chunk_edges(int64_t nnz) {
  int64_t k = 128;
  while (k > 16 && nnz / k < 256 * 64 * 16) k >>= 1;
  return k;
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
