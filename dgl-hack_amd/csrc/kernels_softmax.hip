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
// Row work is cut into fixed chunks of CSR positions (one wave per chunk), rows cut by a chunk boundary are merged in chunk
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

// merge() with one exponential: the larger maximum's own factor is exp(0) = 1.  The
// same (m, l) for finite values; a NaN or +inf anywhere leaves l NaN (so the row's
// softmax is NaN, as with the reference's exp(score - max)); two empty states
// (m = -inf, l = 0) stay empty.
__device__ __forceinline__ void merge1(float& m, float& l, float m2, float l2) {
  const bool ge = m >= m2;
  const float hi = ge ? m : m2, lo = ge ? m2 : m;
  const float lhi = ge ? l : l2, llo = ge ? l2 : l;
  if (hi == -INFINITY) return;
  l = lhi + llo * expf(lo - hi);
  m = hi;
}

// One wave per chunk of K CSR positions, walked L = 64 / H positions at a time with
// lane (j, h) on position base + j and head h: every load instruction reads L
// consecutive positions' row ids and edge ids and, when the edge ids are the
// positions (a position view), one contiguous 256-byte run of logits.  (A lane per
// chunk walking its own positions -- the round-1 form -- kept 64 streams per wave
// whose lines left L2 before the lane came back: 6 ms for 1.4 GB at H = 1.)  The
// positions of one step are reduced by a segmented inclusive scan over j (rows are
// sorted, so equal row ids are one segment); each finished segment is written out,
// the step's last one carries into the next step.  Outputs per chunk as before: a row
// continued from the previous chunk goes to the chunk's carry, every other row to
// the row statistics, and k_sm_fixup merges the carries in chunk order --
// deterministic, no atomics.
template <int H, int MODE>
__global__ void __launch_bounds__(kBlock) k_sm_rows(SoftmaxArgs a) {
  constexpr int L = 64 / H;      // positions per step
  constexpr int U = L >= 16 ? 2 : 4;  // steps whose loads are issued together
  const int lane = threadIdx.x & 63, j = lane / H, h = lane % H;
  const int64_t chunk = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // k_sm_fixup's counters
  const int first_row = a.rows[p0];
  const bool cont = p0 > 0 && a.rows[p0 - 1] == first_row;
  auto put = [&](int row, float m, float l) {
    const bool carry = cont && row == first_row;
    float* pm = carry ? a.carry + chunk * 2 * H : a.stat0 + (int64_t)row * H;
    pm[h] = m;
    if constexpr (MODE == SM_STATS) (carry ? pm + H : a.stat1 + (int64_t)row * H)[h] = l;
  };
  int run_row = -1;  // the row the previous step ended in, and its partial state
  float run_m = MODE == SM_STATS ? -INFINITY : 0.0f, run_l = 0.0f;
  for (int64_t base = p0; base < p1; base += U * L) {
    int r[U];
    float x[U], g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = base + u * L + j;
      r[u] = -1;
      x[u] = MODE == SM_STATS ? -INFINITY : 0.0f;
      g[u] = 0.0f;
      if (p < p1) {
        r[u] = a.rows[p];
        const int64_t e = a.eids[p];
        x[u] = a.s[e * H + h];
        if constexpr (MODE == SM_DOTSUM) g[u] = a.ga[e * H + h];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sb = base + u * L;
      if (sb >= p1) break;  // wave-uniform
      const int jl = p1 - sb < L ? static_cast<int>(p1 - sb) - 1 : L - 1;  // last valid j
      float m, l;
      if constexpr (MODE == SM_STATS) {
        m = x[u];
        l = x[u] == INFINITY ? __builtin_nanf("") : (x[u] == -INFINITY ? 0.0f : 1.0f);
      } else {
        m = x[u] * g[u];
        l = 0.0f;
      }
      // the previous step's last row: continued by this step's first segment, or done
      const int r0 = __shfl(r[u], h);
      if (run_row >= 0) {
        if (r0 == run_row) {
          if (j == 0) {
            if constexpr (MODE == SM_STATS) merge1(m, l, run_m, run_l);
            else m += run_m;
          }
        } else if (j == 0) {
          put(run_row, run_m, run_l);
        }
      }
#pragma unroll
      for (int d = 1; d < L; d <<= 1) {
        const float m2 = __shfl_up(m, d * H);
        const float l2 = MODE == SM_STATS ? __shfl_up(l, d * H) : 0.0f;
        const int r2 = __shfl_up(r[u], d * H);
        if (j >= d && r2 == r[u]) {
          if constexpr (MODE == SM_STATS) merge1(m, l, m2, l2);
          else m += m2;
        }
      }
      const int rn = __shfl_down(r[u], H);
      const int rl = __shfl(r[u], jl * H + h);
      const bool seg_end = j <= jl && (j == jl || rn != r[u]);
      if (seg_end && r[u] != rl) put(r[u], m, l);
      run_row = rl;
      run_m = __shfl(m, jl * H + h);
      run_l = MODE == SM_STATS ? __shfl(l, jl * H + h) : 0.0f;
    }
  }
  if (j == 0) put(run_row, run_m, run_l);
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
  // k_sm_rows: one wave per chunk
  const dim3 rrb(static_cast<unsigned>((chunks + kBlock / 64 - 1) / (kBlock / 64)));
  const int64_t eb = (a.nnz + kBlock - 1) / kBlock;
  const dim3 ebl(static_cast<unsigned>(eb < 256 * 64 ? eb : 256 * 64));
  if (!backward) {
    hipLaunchKernelGGL((k_sm_rows<H, SM_STATS>), rrb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_STATS>), rb, blk, 0, st, a);
    hipLaunchKernelGGL((k_sm_edges<H, SM_NORMALIZE>), ebl, blk, 0, st, a);
  } else {
    hipLaunchKernelGGL((k_sm_rows<H, SM_DOTSUM>), rrb, blk, 0, st, a);
    if (chunks > 1) hipLaunchKernelGGL((k_sm_fixup<H, SM_DOTSUM>), rb, blk, 0, st, a);
    hipLaunchKernelGGL((k_sm_edges<H, SM_GRAD>), ebl, blk, 0, st, a);
  }
}

}  // namespace

bool softmax_supported(int64_t H) { return H == 1 || H == 2 || H == 4 || H == 8 || H == 16; }

// positions per chunk (one wave each): 16 steps of 64 / H positions, fewer while the
// graph would give fewer than 2048 waves
int64_t softmax_chunk_edges(int64_t nnz, int64_t H) {
  const int64_t L = H >= 1 && H <= 64 ? 64 / H : 1;
  int64_t steps = 16;
  while (steps > 1 && nnz / (L * steps) < 2048) steps >>= 1;
  return L * steps;
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
