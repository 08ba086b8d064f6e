// Load-balanced chunk kernels of the g-SpMM family (kernels_spmm.hip has the
// design notes), shared by the translation units that instantiate them: one per
// row slot width (float4 in kernels_spmm.hip, float2 / float in
// kernels_spmm_vw{2,1}.hip), so the three compile in parallel.
#pragma once
#include "internal.h"

#include <climits>
#include <cstdlib>

namespace dglmi {
namespace {

constexpr int kBlock = 256;

// Row slots are VW floats wide: float4 when F % 4 == 0, float2 when F is even,
// single floats otherwise (Reddit's F_in = 602 rows start 8-byte aligned only),
// so a row of any width stays on the load-balanced kernels.
template <int VW> struct VecT;
template <> struct VecT<4> { using T = float4; };
template <> struct VecT<2> { using T = float2; };
template <> struct VecT<1> { using T = float; };

__device__ __forceinline__ float4 ld4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int VW>
__device__ __forceinline__ typename VecT<VW>::T vld(const float* p) {
  return *reinterpret_cast<const typename VecT<VW>::T*>(p);
}
template <int VW>
__device__ __forceinline__ typename VecT<VW>::T vld_nt(const float* p) {
  if constexpr (VW == 4) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else if constexpr (VW == 2) {
    const f32x2 v = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(p));
    return make_float2(v.x, v.y);
  } else {
    return __builtin_nontemporal_load(p);
  }
}
__device__ __forceinline__ void vst(float* p, float4 v) { st4(p, v); }
__device__ __forceinline__ void vst(float* p, float2 v) { *reinterpret_cast<float2*>(p) = v; }
__device__ __forceinline__ void vst(float* p, float v) { *p = v; }
__device__ __forceinline__ void vst_nt(float* p, float4 v) {
  __builtin_nontemporal_store(v.x, p);
  __builtin_nontemporal_store(v.y, p + 1);
  __builtin_nontemporal_store(v.z, p + 2);
  __builtin_nontemporal_store(v.w, p + 3);
}
__device__ __forceinline__ void vst_nt(float* p, float2 v) {
  __builtin_nontemporal_store(v.x, p);
  __builtin_nontemporal_store(v.y, p + 1);
}
__device__ __forceinline__ void vst_nt(float* p, float v) { __builtin_nontemporal_store(v, p); }

template <int RED>
__device__ __forceinline__ float4 vred(float4 a, float4 b) {
  return make_float4(red_apply<RED>(a.x, b.x), red_apply<RED>(a.y, b.y),
                     red_apply<RED>(a.z, b.z), red_apply<RED>(a.w, b.w));
}
template <int RED>
__device__ __forceinline__ float2 vred(float2 a, float2 b) {
  return make_float2(red_apply<RED>(a.x, b.x), red_apply<RED>(a.y, b.y));
}
template <int RED>
__device__ __forceinline__ float vred(float a, float b) { return red_apply<RED>(a, b); }
template <int VW, int RED>
__device__ __forceinline__ typename VecT<VW>::T vident() {
  const float v = red_identity<RED>();
  if constexpr (VW == 4) return make_float4(v, v, v, v);
  else if constexpr (VW == 2) return make_float2(v, v);
  else return v;
}
template <int VW>
__device__ __forceinline__ typename VecT<VW>::T vone() {
  if constexpr (VW == 4) return make_float4(1.0f, 1.0f, 1.0f, 1.0f);
  else if constexpr (VW == 2) return make_float2(1.0f, 1.0f);
  else return 1.0f;
}
__device__ __forceinline__ float4 vscale(float4 a, float m) { return make_float4(a.x * m, a.y * m, a.z * m, a.w * m); }
__device__ __forceinline__ float2 vscale(float2 a, float m) { return make_float2(a.x * m, a.y * m); }
__device__ __forceinline__ float vscale(float a, float m) { return a * m; }
__device__ __forceinline__ float4 vdivs(float4 a, float d) { return make_float4(a.x / d, a.y / d, a.z / d, a.w / d); }
__device__ __forceinline__ float2 vdivs(float2 a, float d) { return make_float2(a.x / d, a.y / d); }
__device__ __forceinline__ float vdivs(float a, float d) { return a / d; }
__device__ __forceinline__ float4 vadd(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float2 vadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ float4 vmul(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
__device__ __forceinline__ float2 vmul(float2 a, float2 b) { return make_float2(a.x * b.x, a.y * b.y); }
__device__ __forceinline__ float vmul(float a, float b) { return a * b; }
// where(a == b, g, 0) per component: the max / min gradient's tie mask
__device__ __forceinline__ float vtie(float a, float b, float g) { return a == b ? g : 0.0f; }
__device__ __forceinline__ float2 vtie(float2 a, float2 b, float2 g) {
  return make_float2(vtie(a.x, b.x, g.x), vtie(a.y, b.y, g.y));
}
__device__ __forceinline__ float4 vtie(float4 a, float4 b, float4 g) {
  return make_float4(vtie(a.x, b.x, g.x), vtie(a.y, b.y, g.y), vtie(a.z, b.z, g.z), vtie(a.w, b.w, g.w));
}

// VAR bit 15: gathers by raw buffer loads, cold (bit-31-marked) rows with aux
// policy (VAR >> 5) & 31, the others with (VAR >> 10) & 31 (aux: 1 = sc0,
// 2 = nt, 16 = sc1) -- the cache-policy probe's variants.
constexpr int kVarBuf = 1 << 15;
constexpr int var_pol(int hot_aux, int cold_aux) { return 11 | kVarBuf | (cold_aux << 5) | (hot_aux << 10); }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int AUX>
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, AUX);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}

template <int KIND>
constexpr bool needs_eid() {
  return KIND != FAST_COPY_COL && KIND != FAST_COL_TIE && KIND != FAST_COL_MUL_POS;
}

// Value of one edge for VW-float slot fv of the output row.  `hs` (bcast kind):
// the edge value's index for this slot, (VW * fv) / head_dim, and `wn` the edge
// values per edge, F / head_dim -- both hoisted out of the edge loop by the
// caller (64-bit divisions per edge cost 1.7 ms on the C5 typed gather).
template <int KIND, int VW>
__device__ __forceinline__ typename VecT<VW>::T edge_value(const FastArgs& a, int32_t col, int64_t eid,
                                                          int fv, int hs = 0, int64_t wn = 1,
                                                          int32_t row = 0) {
  if constexpr (KIND == FAST_COL_TIE) {
    // grad_x[row] += grad_out[col] where x[row] == out[col] (the reference's
    // BackwardCall for max / min: every tied edge gets the gradient)
    const int64_t o = static_cast<int64_t>(col) * a.F + VW * fv;
    return vtie(vld<VW>(a.xr + static_cast<int64_t>(row) * a.F + VW * fv), vld<VW>(a.w + o),
                vld<VW>(a.x + o));
  } else if constexpr (KIND == FAST_COPY_COL) {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    return vld<VW>(a.x + c * a.F + VW * fv);
  } else if constexpr (KIND == FAST_COPY_EDGE) {
    const int64_t e = a.x_map ? a.x_map[eid] : eid;
    return vld<VW>(a.x + e * a.F + VW * fv);
  } else if constexpr (KIND == FAST_COL_MUL_EDGE) {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    const int64_t e = a.w_map ? a.w_map[eid] : eid;
    return vmul(vld<VW>(a.x + c * a.F + VW * fv), vld<VW>(a.w + e * a.F + VW * fv));
  } else if constexpr (KIND == FAST_COL_MUL_POS) {
    // the position's weight is staged with the walk (s_w) and applied by the caller;
    // there is no edge id to index the weight by
    const int64_t c = a.x_map ? a.x_map[col] : col;
    return vld<VW>(a.x + c * a.F + VW * fv);
  } else {
    const int64_t c = a.x_map ? a.x_map[col] : col;
    const int64_t e = a.w_map ? a.w_map[eid] : eid;
    return vscale(vld<VW>(a.x + c * a.F + VW * fv), a.w[e * wn + hs]);
  }
}

template <int VAR>
__device__ __forceinline__ int32_t ld_stream(const int32_t* p) {
  if constexpr (VAR & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int VAR>
__device__ __forceinline__ int64_t ld_stream(IdxPtr q, int64_t p) {
  if (q.wide) {
    const int64_t* x = static_cast<const int64_t*>(q.p) + p;
    if constexpr (VAR & 1) return __builtin_nontemporal_load(x);
    else return *x;
  }
  return ld_stream<VAR>(static_cast<const int32_t*>(q.p) + p);
}
template <int VAR>
__device__ __forceinline__ float ld_stream_f(const float* p) {
  if constexpr (VAR & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int VAR, typename V>
__device__ __forceinline__ void st_out(float* p, V v) {
  if constexpr (VAR & 2) vst_nt(p, v);
  else vst(p, v);
}

// L lanes per group, NV VW-float slots per lane, U gathers in flight per lane-slot.
// VAR (tuning variants): bit 0 non-temporal index/row stream loads, bit 1
// non-temporal output stores, bit 2 twice the gathers in flight.  Default 3:
// keeping the once-read CSR stream and the once-written output out of L2/MALL
// leaves more room for re-read source rows (M1: 3.30 -> 3.25 ms; 4 and 7 spill).
// EPI: fused epilogue on every finished row, out = acc * row_mul[r] / row_div[r]
// + bias + addend[r] (GraphConv's norm and bias, the mean reducer's division,
// accumulation onto an earlier partial result) -- applied
// once per row, after the whole row is reduced (split rows: in the fixup).
template <bool EPI, int VW>
__device__ __forceinline__ typename VecT<VW>::T epiv(const FastArgs& a, typename VecT<VW>::T v,
                                                    int64_t r, int fv) {
  if constexpr (EPI) {
    if (a.row_mul) v = vscale(v, a.row_mul[r]);
    if (a.row_div) v = vdivs(v, a.row_div[r]);
    if (a.bias) v = vadd(v, vld<VW>(a.bias + VW * fv));
    if (a.addend) v = vadd(v, vld<VW>(a.addend + r * a.F + VW * fv));
  }
  return v;
}

template <int KIND, int RED, int L, int NV, int VAR = 3, bool EPI = false, int VW = 4>
__global__ void __launch_bounds__(kBlock) k_chunk_reduce(FastArgs a, IdxPtr indptr) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront (fill_empty_rows)");
  constexpr int G = kBlock / L;           // groups per block
  constexpr int B = (L > 16 ? L : 16) * ((VAR & 4) ? 2 : 1);  // positions staged per step
  constexpr int U = (NV == 1 ? 8 : (NV == 2 ? 4 : 2)) * ((VAR & 4) ? 2 : 1);
  static_assert(B % U == 0, "B must be a multiple of U");
  __shared__ int32_t s_row[G][B];
  __shared__ int32_t s_col[G][B];
  __shared__ int64_t s_eid[needs_eid<KIND>() ? G : 1][needs_eid<KIND>() ? B : 1];
  // FAST_COL_MUL_POS: one scalar edge value per position (u_mul_e with one weight per
  // edge, edge ids = the positions of a position view), staged with the rows and
  // columns by one coalesced load instead of a per-lane load behind a staged edge id
  constexpr bool kScalarW = KIND == FAST_COL_MUL_POS;
  __shared__ float s_w[kScalarW ? G : 1][kScalarW ? B : 1];

  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;  // whole group exits together
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // k_chunk_fixup's counters
  using V = typename VecT<VW>::T;
  const int F4 = static_cast<int>(a.F / VW);
  const V I = vident<VW, RED>();
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, -1, 0x00020000);
  int hsel[NV];  // bcast: edge value index of each slot
  const int64_t wn = KIND == FAST_COL_MUL_EDGE_BCAST ? a.F / a.head_dim : 1;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    hsel[v] = KIND == FAST_COL_MUL_EDGE_BCAST ? static_cast<int>((VW * (lane + v * L)) / a.head_dim) : 0;

  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  V acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = I;

  // B positions per batch staged through LDS (coalesced, one row/col/eid per lane slot);
  // each batch's ids are loaded into registers one batch ahead, while the previous
  // batch's gathers are in flight, and written to LDS at the batch's start
  constexpr int SQ = B / L;  // positions each lane stages per batch
  constexpr bool kEid = needs_eid<KIND>();
  int32_t nr[SQ], nc[SQ];
  [[maybe_unused]] int64_t ne[kEid ? SQ : 1];
  [[maybe_unused]] float nw[kScalarW ? SQ : 1];
  auto fetch = [&](int64_t nb) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int64_t p = nb + lane + i * L;
      const bool ok = p < p1;
      nr[i] = ok ? ld_stream<VAR>(a.rows + p) : INT_MAX;
      nc[i] = ok ? ld_stream<VAR>(a.indices + p) : 0;
      // identity edge ids (a position view's walk, a.eids null): no `data` stream
      if constexpr (kEid) ne[kEid ? i : 0] = ok ? (a.eids ? ld_stream<VAR>(a.eids, p) : p) : 0;
      if constexpr (kScalarW) nw[kScalarW ? i : 0] = ok ? ld_stream_f<VAR>(a.w + p) : 0.0f;
    }
  };
  fetch(p0);
  for (int64_t base = p0; base < p1; base += B) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int q = lane + i * L;
      s_row[g][q] = nr[i];
      s_col[g][q] = nc[i];
      if constexpr (kEid) s_eid[kEid ? g : 0][q] = ne[kEid ? i : 0];
      if constexpr (kScalarW) s_w[kScalarW ? g : 0][kScalarW ? q : 0] = nw[kScalarW ? i : 0];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (base + B < p1) fetch(base + B);
    // the mul kinds load both operands in the gather loop and multiply in the
    // accumulation loop: a product inside the bounds-checked gather made the compiler
    // wait for each gather before issuing the next (s_waitcnt vmcnt(0) per edge)
    constexpr bool kMulVec = KIND == FAST_COL_MUL_EDGE;
    constexpr bool kMulScl = KIND == FAST_COL_MUL_EDGE_BCAST || KIND == FAST_COL_MUL_POS;
    // the max / min gradient: both gathered rows first, the tie test (against the
    // walk row's own value) in the accumulation loop
    constexpr bool kTie = KIND == FAST_COL_TIE;
    constexpr bool kTwo = kMulVec || kTie;  // a second gathered row per edge
#pragma unroll
    for (int ub = 0; ub < B; ub += U) {
      V val[U][NV];
      [[maybe_unused]] V wv[kTwo ? U : 1][kTwo ? NV : 1];
      [[maybe_unused]] float wsc[kMulScl ? U : 1][kMulScl ? NV : 1];
      bool fast_mul = false;
      if constexpr (kMulVec || kMulScl || kTie) fast_mul = a.x_map == nullptr && a.w_map == nullptr;
      if (fast_mul) {
        if constexpr (kMulVec || kMulScl || kTie) {
        // (sum only: I = 0; positions past the chunk are never accumulated; no maps:
        // a map load in flight made the compiler wait for every earlier gather)
        // every gather first, then the weights
        int64_t cc[U], ee[U];
        bool okk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cc[u] = s_col[g][ub + u];
          okk[u] = s_row[g][ub + u] != INT_MAX;
          if constexpr (!kScalarW && !kTie) ee[u] = s_eid[needs_eid<KIND>() ? g : 0][ub + u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int f4 = lane + v * L;
            val[u][v] = (okk[u] && f4 < F4) ? vld<VW>(a.x + cc[u] * a.F + VW * f4) : I;
          }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int f4 = lane + v * L;
            const bool in = okk[u] && f4 < F4;
            if constexpr (kScalarW)
              wsc[u][kMulScl ? v : 0] = s_w[kScalarW ? g : 0][kScalarW ? ub + u : 0];
            else if constexpr (kMulScl)
              wsc[u][kMulScl ? v : 0] = in ? a.w[ee[u] * wn + hsel[v]] : 0.0f;
            else if constexpr (kTie)
              wv[kTwo ? u : 0][kTwo ? v : 0] = in ? vld<VW>(a.w + cc[u] * a.F + VW * f4) : I;
            else
              wv[kTwo ? u : 0][kTwo ? v : 0] = in ? vld<VW>(a.w + ee[u] * a.F + VW * f4) : I;
          }
        }
      } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t col = s_col[g][ub + u];
        const int64_t eid = needs_eid<KIND>() ? s_eid[needs_eid<KIND>() ? g : 0][ub + u] : 0;
        const bool ok = s_row[g][ub + u] != INT_MAX;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int f4 = lane + v * L;
          if constexpr ((VAR & kVarBuf) != 0 && KIND == FAST_COPY_COL && VW == 4) {
            // cache-policy probe (scripts/policy_probe.py): marked / unmarked rows
            // gathered by buffer loads with the aux policies encoded in VAR
            // (table < 4 GiB: 32-bit byte offsets, checked by the launcher)
            const bool cold = col < 0;
            const uint32_t off = (static_cast<uint32_t>(col & 0x7fffffff) * static_cast<uint32_t>(a.F) +
                                  static_cast<uint32_t>(VW * f4)) * 4u;
            if (ok && f4 < F4)
              val[u][v] = cold ? buf_ld4<(VAR >> 5) & 31>(rsrc, off) : buf_ld4<(VAR >> 10) & 31>(rsrc, off);
            else
              val[u][v] = I;
          } else if constexpr ((VAR & 8) != 0 && KIND == FAST_COPY_COL) {
            // bit 31 of the column marks a cold source row (re-read fewer than
            // min_hot_degree times): gathered non-temporally so it does not evict
            // re-read rows from L2 / Infinity Cache (VAR & 16: the reverse, a
            // tuning control)
            const bool nt = (col < 0) != ((VAR & 16) != 0);
            const float* px = a.x + static_cast<int64_t>(col & 0x7fffffff) * a.F + VW * f4;
            val[u][v] = (ok && f4 < F4) ? (nt ? vld_nt<VW>(px) : vld<VW>(px)) : I;
          } else {
            val[u][v] = (ok && f4 < F4) ? edge_value<KIND, VW>(a, col, eid, f4, hsel[v], wn, s_row[g][ub + u]) : I;
            // (mapped mul kinds: the product is already in val, except the staged
            // per-position weight)
            if constexpr (kScalarW) wsc[u][kMulScl ? v : 0] = s_w[kScalarW ? g : 0][kScalarW ? ub + u : 0];
            else if constexpr (kMulScl) wsc[u][kMulScl ? v : 0] = 1.0f;
            if constexpr (kMulVec) wv[kTwo ? u : 0][kTwo ? v : 0] = vone<VW>();
          }
        }
      }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t r = s_row[g][ub + u];
        if (r == INT_MAX) break;
        if (r != cur) {
          // flush the finished row (empty rows in between: fill_empty_rows)
          float* dst = cont ? a.carry + chunk * a.F : a.out + cur * a.F;
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int f4 = lane + v * L;
            if (f4 < F4) st_out<VAR>(dst + VW * f4, cont ? acc[v] : epiv<EPI, VW>(a, acc[v], cur, f4));
            acc[v] = I;
          }
          cur = r;
          cont = false;
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          if constexpr (kMulVec) acc[v] = vred<RED>(acc[v], vmul(val[u][v], wv[kTwo ? u : 0][kTwo ? v : 0]));
          else if constexpr (kTie) {
            // (mapped fallback: val already holds the masked value)
            const int f4 = lane + v * L;
            acc[v] = vred<RED>(acc[v], fast_mul && f4 < F4
                                           ? vtie(vld<VW>(a.xr + static_cast<int64_t>(r) * a.F + VW * f4),
                                                  wv[kTwo ? u : 0][kTwo ? v : 0], val[u][v])
                                           : val[u][v]);
          }
          else if constexpr (kMulScl) acc[v] = vred<RED>(acc[v], vscale(val[u][v], wsc[u][kMulScl ? v : 0]));
          else acc[v] = vred<RED>(acc[v], val[u][v]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  {
    float* dst = cont ? a.carry + chunk * a.F : a.out + cur * a.F;
    // a row that goes on in the next chunk stays raw: the fixup finishes it
    const bool done = !cont && !(EPI && p1 < a.nnz && a.rows[p1] == cur);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      if (f4 < F4) st_out<VAR>(dst + VW * f4, done ? epiv<EPI, VW>(a, acc[v], cur, f4) : acc[v]);
    }
  }
  fill_empty_rows(indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, L, lane, [&](int64_t r) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      if (f4 < F4) st_out<VAR>(a.out + r * a.F + VW * f4, epiv<EPI, VW>(a, I, r, f4));
    }
  });
}

// Fold the carries of every row cut by chunk boundaries into its head, in
// chunk order.  One group per chunk; a row's first continuation chunk does the
// work, or -- for rows of more than kFixSeg continuation chunks, when the
// workspace has counters -- every kFixSeg-th one folds a segment and the last
// to finish folds the head and the segment partials (internal.h).
template <int RED, int L, int NV, bool EPI = false, int VW = 4>
__global__ void __launch_bounds__(kBlock) k_chunk_fixup(FastArgs a, IdxPtr indptr) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront (seg_arrive_last)");
  constexpr int G = kBlock / L;
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (chunk == 0 || p0 >= a.nnz) return;
  const int64_t r = a.rows[p0];
  const int64_t start = indptr[r];
  if (start >= p0) return;  // not a continuation
  const int64_t first = start / K + 1;  // the row's first continuation chunk
  const int64_t last = (indptr[r + 1] - 1) / K;
  const int64_t nseg = a.seg_cnt != nullptr ? (last - first + kFixSeg) / kFixSeg : 1;
  if (nseg == 1 ? chunk != first : (chunk - first) % kFixSeg != 0) return;
  const int64_t cend = nseg == 1 ? last : (chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last);
  using V = typename VecT<VW>::T;
  const int F4 = static_cast<int>(a.F / VW);
  auto fold = [&](V (&acc)[NV], int64_t c0, int64_t c1, int64_t step) {
    int64_t c = c0;
    for (; c + 3 * step <= c1; c += 4 * step) {
      V t[4][NV];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int f4 = lane + v * L;
          t[k][v] = f4 < F4 ? vld<VW>(a.carry + (c + k * step) * a.F + VW * f4) : vident<VW, RED>();
        }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = vred<RED>(acc[v], t[k][v]);
    }
    for (; c <= c1; c += step)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int f4 = lane + v * L;
        if (f4 < F4) acc[v] = vred<RED>(acc[v], vld<VW>(a.carry + c * a.F + VW * f4));
      }
  };
  V acc[NV];
  if (nseg > 1) {
    // this segment's partial, into its own first carry record (already read)
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = vident<VW, RED>();
    fold(acc, chunk, cend, 1);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      if (f4 < F4) vst(a.carry + chunk * a.F + VW * f4, acc[v]);
    }
    if (!seg_arrive_last(a.seg_cnt + first, nseg, L, lane)) return;
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    acc[v] = f4 < F4 ? vld<VW>(a.out + r * a.F + VW * f4) : vident<VW, RED>();
  }
  if (nseg > 1) fold(acc, first, first + (nseg - 1) * kFixSeg, kFixSeg);
  else fold(acc, first, last, 1);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    if (f4 < F4) vst(a.out + r * a.F + VW * f4, epiv<EPI, VW>(a, acc[v], r, f4));
  }
}


// ---------------------------------------------------------------------------
// Narrow rows (F < 16 floats: attention logits per head, edge-softmax sums):
// a group of 4+ lanes would idle most lanes, so ONE lane owns a chunk and the
// whole (tiny) row, keeping 8 gathers of F floats in flight per lane.
inline bool has_epi(const FastArgs& a) { return a.row_mul || a.row_div || a.bias || a.addend; }

struct Cfg {
  int L, NV;
};
// Lanes per group and slots per lane for rows of `slots` VW-float slots.
inline Cfg pick(int64_t slots, int vw) {
  if (vw == 4) {
    if (slots <= 4) return {4, 1};
    if (slots <= 8) return {8, 1};
  }
  if (slots <= 16) return {16, 1};
  if (slots <= 32) return {32, 1};
  if (slots <= 64) return {64, 1};
  if (slots <= 128) return {64, 2};
  if (slots <= 256) return {64, 4};
  if (slots <= 512) return {64, 8};
  return {64, 16};
}

#if DGLMI_PROBES
// Probe build only (`make PROBES=1` -> libdglmi_probes.so): the cache-policy and
// tuning variants of the headline kernel, picked per launch from the
// environment by scripts/policy_probe.py and scripts/tune_spmm.py.  The shipped
// library instantiates only the variants the dispatcher below picks and reads
// no environment on the launch path.
inline int spmm_policy() {
  const char* env = std::getenv("DGLMI_SPMM_POLICY");
  return env ? std::atoi(env) : 0;
}

inline int spmm_variant() {
  const char* env = std::getenv("DGLMI_SPMM_VARIANT");
  return env ? std::atoi(env) : 3;
}
#endif

template <int KIND, int RED, int L, int NV, int VW>
void run(const FastArgs& a, IdxPtr indptr, hipStream_t s) {
  constexpr int G = kBlock / L;
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = static_cast<unsigned>((chunks + G - 1) / G);
  if constexpr (KIND == FAST_COPY_COL && RED == RED_SUM && NV == 1 && L >= 16 && VW == 4) {
    if (a.marked) {  // cold-row hints present (capi.cpp run_fast decides)
#if DGLMI_PROBES
      const int pol = spmm_policy();
      if (pol > 0 && !has_epi(a) && a.num_cols * a.F * 4 <= (int64_t)UINT32_MAX) {
        switch (pol) {
#define DGLMI_POL(K_, H_, C_)                                                                    \
  case K_:                                                                                     \
    hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, var_pol(H_, C_)>), dim3(blocks),      \
                       dim3(kBlock), 0, s, a, indptr);                                         \
    break;
          DGLMI_POL(1, 0, 2) DGLMI_POL(2, 0, 16) DGLMI_POL(3, 0, 17) DGLMI_POL(4, 0, 18)
          DGLMI_POL(5, 0, 3) DGLMI_POL(6, 1, 2) DGLMI_POL(7, 16, 2) DGLMI_POL(8, 0, 0)
          DGLMI_POL(9, 2, 2)
#undef DGLMI_POL
          default: break;
        }
        if (chunks > 1)
          hipLaunchKernelGGL((k_chunk_fixup<RED, L, NV>), dim3(blocks), dim3(kBlock), 0, s, a, indptr);
        return;
      }
#endif
      if (has_epi(a))
        hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 11, true>), dim3(blocks), dim3(kBlock),
                           0, s, a, indptr);
      else
        hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 11>), dim3(blocks), dim3(kBlock), 0, s,
                           a, indptr);
      if (chunks > 1) {
        if (has_epi(a))
          hipLaunchKernelGGL((k_chunk_fixup<RED, L, NV, true>), dim3(blocks), dim3(kBlock), 0, s, a,
                             indptr);
        else
          hipLaunchKernelGGL((k_chunk_fixup<RED, L, NV>), dim3(blocks), dim3(kBlock), 0, s, a,
                             indptr);
      }
      return;
    }
  }
  if constexpr (RED == RED_SUM) {
    if (has_epi(a)) {
      hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 3, true, VW>), dim3(blocks), dim3(kBlock),
                         0, s, a, indptr);
      if (chunks > 1)
        hipLaunchKernelGGL((k_chunk_fixup<RED, L, NV, true, VW>), dim3(blocks), dim3(kBlock), 0, s, a,
                           indptr);
      return;
    }
  }
#if DGLMI_PROBES
  if constexpr (KIND == FAST_COPY_COL && RED == RED_SUM && L == 16 && NV == 1 && VW == 4) {
    // tuning variants of the headline kernel (scripts/tune_spmm.py)
    switch (spmm_variant()) {
      case 0: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 0>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 1: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 1>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 2: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 2>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 4: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 4>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 7: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 7>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 27: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 27>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      default: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
    }
  } else if constexpr (KIND == FAST_COL_MUL_EDGE_BCAST && RED == RED_SUM && L == 16 && NV == 1 &&
                       VW == 4) {
    // the same variants for u_mul_e_sum with a per-head edge weight (GAT composition)
    switch (spmm_variant()) {
      case 0: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 0>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 1: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 1>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      case 7: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 7>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
      default: hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV>), dim3(blocks), dim3(kBlock), 0, s, a, indptr); break;
    }
  } else
#endif
  {
    hipLaunchKernelGGL((k_chunk_reduce<KIND, RED, L, NV, 3, false, VW>), dim3(blocks), dim3(kBlock),
                       0, s, a, indptr);
  }
  if (chunks > 1)
    hipLaunchKernelGGL((k_chunk_fixup<RED, L, NV, false, VW>), dim3(blocks), dim3(kBlock), 0, s, a,
                       indptr);
}

// Widest slot (4, 2 or 1 floats) dividing the row -- and, for the broadcast
// kind, the head width, so one slot never spans two edge values.
inline int fast_vw(int64_t F, int kind, int64_t head_dim) {
  for (int vw = 4; vw > 1; vw >>= 1)
    if (F % vw == 0 && (kind != FAST_COL_MUL_EDGE_BCAST || head_dim % vw == 0)) return vw;
  return 1;
}

inline bool lane_kernel_width(int64_t F) { return F >= 1 && (F <= 8 || F == 12); }

template <int KIND, int RED, int VW>
void run_vw(const FastArgs& a, IdxPtr indptr, hipStream_t s) {
  const Cfg c = pick(a.F / VW, VW);
  switch (c.L * 10 + c.NV) {
    case 41: if constexpr (VW == 4) run<KIND, RED, 4, 1, VW>(a, indptr, s); break;
    case 81: if constexpr (VW == 4) run<KIND, RED, 8, 1, VW>(a, indptr, s); break;
    case 161: run<KIND, RED, 16, 1, VW>(a, indptr, s); break;
    case 321: run<KIND, RED, 32, 1, VW>(a, indptr, s); break;
    case 641: run<KIND, RED, 64, 1, VW>(a, indptr, s); break;
    case 642: run<KIND, RED, 64, 2, VW>(a, indptr, s); break;
    case 644: run<KIND, RED, 64, 4, VW>(a, indptr, s); break;
    case 648: run<KIND, RED, 64, 8, VW>(a, indptr, s); break;
    default: if constexpr (VW != 4) run<KIND, RED, 64, 16, VW>(a, indptr, s); break;
  }
}
}  // namespace

// Chunk-kernel reduce for rows of float2 (vw2) / single-float (vw1) slots.
void launch_fast_chunk_vw2(int kind, int red, const FastArgs& a, hipStream_t s);
void launch_fast_chunk_vw1(int kind, int red, const FastArgs& a, hipStream_t s);

}  // namespace dglmi
