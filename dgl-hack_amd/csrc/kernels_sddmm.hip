// Per-edge outputs (g-SDDMM) for gfx950: apply_edges with the builtin binary
// message functions (u_add_v, u_dot_v, e_sub_v, e_div_v, u_mul_e, ...; reducer
// "none") and the per-edge gradients of every binary op.
//
// Reference: the per-edge UDF of cpu/binary_reduce_impl.h:29-52 with
// ReduceNone (cpu/functor.h:63-71: out[eid] = op(lhs, rhs)), BinaryDot
// (binary_reduce_common.h:196-213) and the edge branch of the backward UDF
// (cpu/backward_binary_reduce_impl.h:39-83); on GPU the reference runs the
// same minigun edge-parallel kernel as for reductions, one thread per
// (edge, feature) with a binary search for the source row.
//
// Design (MI355X-first):
//  * Items are edges in EDGE-ID order when the graph supplies its COO
//    (DGLMIGraph.coo_src/coo_dst): outputs and edge operands stream
//    sequentially and only node operands are gathered.  Without it (parent-eid
//    subgraphs) items are in-CSR positions and outputs are scattered by eid.
//  * Narrow rows (<= 8 floats per operand: attention logits per head, softmax
//    terms) use one lane per edge with the whole row in registers, 64 edges per
//    wavefront in flight.  Wider rows use a group of L lanes per edge with
//    float4 slices; dot products reduce their float4 partials with cross-lane
//    xor shuffles inside the group.
//  * Every output element is written exactly once; no atomics, no fill pass.
#include "internal.h"

namespace dglmi {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

template <int NF>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[NF]) {
  if constexpr (NF % 4 == 0) {
#pragma unroll
    for (int i = 0; i < NF / 4; ++i) {
      const float4 t = ld4(p + 4 * i);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else if constexpr (NF % 2 == 0) {
#pragma unroll
    for (int i = 0; i < NF / 2; ++i) {
      const float2 t = *reinterpret_cast<const float2*>(p + 2 * i);
      v[2 * i] = t.x; v[2 * i + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < NF; ++i) v[i] = p[i];
  }
}

template <int NF>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[NF]) {
  if constexpr (NF % 4 == 0) {
#pragma unroll
    for (int i = 0; i < NF / 4; ++i) st4(p + 4 * i, make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]));
  } else if constexpr (NF % 2 == 0) {
#pragma unroll
    for (int i = 0; i < NF / 2; ++i) *reinterpret_cast<float2*>(p + 2 * i) = make_float2(v[2 * i], v[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < NF; ++i) p[i] = v[i];
  }
}

__device__ __forceinline__ int64_t pick(int role, int64_t row, int64_t col, int64_t eid) {
  return role == ROLE_ROW ? row : (role == ROLE_COL ? col : (role == ROLE_EDGE ? eid : 0));
}

template <int OP>
__device__ __forceinline__ float op1(float l, float r) {
  if constexpr (OP == OP_ADD) return l + r;
  else if constexpr (OP == OP_SUB) return l - r;
  else if constexpr (OP == OP_MUL) return l * r;
  else if constexpr (OP == OP_DIV) return l / r;
  else return l;
}

// Which operand rows the gradient wrt operand `want` reads.
template <int OP>
__device__ __forceinline__ bool bwd_needs_lhs(int want) {
  return (OP == OP_MUL || OP == OP_DOT || OP == OP_DIV) && want == 1;
}
template <int OP>
__device__ __forceinline__ bool bwd_needs_rhs(int want) {
  return (OP == OP_MUL || OP == OP_DOT || OP == OP_DIV);
}
template <int OP>
__device__ __forceinline__ float bwd1(float ge, float l, float r, int want) {
  if constexpr (OP == OP_USE_LHS) return ge;
  else return want == 0 ? ge * op_grad_lhs<OP>(l, r) : ge * op_grad_rhs<OP>(l, r);
}

__device__ __forceinline__ void item(const SddmmArgs& a, int64_t p, int64_t& row, int64_t& col,
                                     int64_t& eid) {
  row = a.rows[p];
  col = a.cols[p];
  eid = a.eids ? a.eids[p] : p;
}

// ---- one lane per edge (NF <= 8 floats per operand row) ---------------------
template <int OP, bool BWD, int NF>
__global__ void __launch_bounds__(kBlock) k_sddmm_lane(SddmmArgs a) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t len = a.len;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < a.nnz; p += stride) {
    int64_t row, col, eid;
    item(a, p, row, col, eid);
    float l[NF], r[NF];
    const bool need_l = !BWD || bwd_needs_lhs<OP>(a.want);
    const bool need_r = OP != OP_USE_LHS && (!BWD || bwd_needs_rhs<OP>(a.want));
    if (need_l) load_row<NF>(a.lhs + pick(a.lhs_role, row, col, eid) * NF, l);
    else {
#pragma unroll
      for (int i = 0; i < NF; ++i) l[i] = 0.0f;
    }
    if (need_r) load_row<NF>(a.rhs + pick(a.rhs_role, row, col, eid) * NF, r);
    else {
#pragma unroll
      for (int i = 0; i < NF; ++i) r[i] = 0.0f;
    }
    if constexpr (!BWD) {
      if constexpr (OP == OP_DOT) {
        // sequential per segment, the order of BinaryDot (binary_reduce_common.h:196-213)
        const int64_t D = NF / len;
        float* o = a.out + eid * D;
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          acc = ((i % len) == 0 ? 0.0f : acc) + l[i] * r[i];
          if ((i % len) == len - 1) o[i / len] = acc;
        }
      } else {
        float o[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) o[i] = op1<OP>(l[i], r[i]);
        store_row<NF>(a.out + eid * NF, o);
      }
    } else {
      const int64_t D = NF / len;
      const float* go = a.go + pick(a.go_role, row, col, eid) * D;
      float g[NF];
      if (OP == OP_DOT && len > 1) {
#pragma unroll
        for (int i = 0; i < NF; ++i) g[i] = bwd1<OP>(go[i / len], l[i], r[i], a.want);
      } else {
        float gv[NF];
        load_row<NF>(go, gv);
#pragma unroll
        for (int i = 0; i < NF; ++i) g[i] = bwd1<OP>(gv[i], l[i], r[i], a.want);
      }
      store_row<NF>(a.out + eid * NF, g);
    }
  }
}

// ---- a group of L lanes per edge, float4 slices (NF % 4 == 0, NF >= 16) -----
// A group takes U consecutive items per iteration: their ids, then every operand load,
// then the outputs, so U edges' gathers are in flight per group (one edge at a time:
// C3 u_dot_v(ft, grad) for the GAT composition's attention gradient, 16 lanes per edge,
// 6.69 ms).
template <int NV>
struct GroupUnroll {
  static constexpr int U = NV == 1 ? 4 : (NV == 2 ? 2 : 1);
};

template <int OP, bool BWD, int L, int NV>
__global__ void __launch_bounds__(kBlock) k_sddmm_group(SddmmArgs a) {
  constexpr int G = kBlock / L;
  constexpr int U = GroupUnroll<NV>::U;
  const int lane = threadIdx.x % L;
  const int64_t NF = a.D * a.len;
  const int NF4 = static_cast<int>(NF / 4);
  const int64_t len = a.len;
  const int S = static_cast<int>(len / 4);  // float4 per dot segment (pow2)
  const int64_t stride = (int64_t)gridDim.x * G * U;
  const bool need_l = !BWD || bwd_needs_lhs<OP>(a.want);
  const bool need_r = OP != OP_USE_LHS && (!BWD || bwd_needs_rhs<OP>(a.want));
  for (int64_t p0 = ((int64_t)blockIdx.x * G + threadIdx.x / L) * U; p0 < a.nnz; p0 += stride) {
    int64_t row[U], col[U], eid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + u < a.nnz ? p0 + u : a.nnz - 1;
      item(a, p, row[u], col[u], eid[u]);
    }
    float4 l4[U][NV], r4[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* lp = a.lhs + pick(a.lhs_role, row[u], col[u], eid[u]) * NF;
      const float* rp = need_r ? a.rhs + pick(a.rhs_role, row[u], col[u], eid[u]) * NF : nullptr;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int f4 = lane + v * L;
        const bool ok = f4 < NF4 && p0 + u < a.nnz;
        l4[u][v] = (ok && need_l) ? ld4(lp + 4 * f4) : make_float4(0.f, 0.f, 0.f, 0.f);
        r4[u][v] = (ok && need_r) ? ld4(rp + 4 * f4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p0 + u >= a.nnz) break;
      if constexpr (!BWD) {
        if constexpr (OP == OP_DOT) {
          float part[NV];
#pragma unroll
          for (int v = 0; v < NV; ++v)
            part[v] = ((l4[u][v].x * r4[u][v].x + l4[u][v].y * r4[u][v].y) + l4[u][v].z * r4[u][v].z) +
                      l4[u][v].w * r4[u][v].w;
          const int span = S < L ? S : L;
          for (int o = 1; o < span; o <<= 1) {
#pragma unroll
            for (int v = 0; v < NV; ++v) part[v] += __shfl_xor(part[v], o, L);
          }
          float* out = a.out + eid[u] * a.D;
          if (S <= L) {
#pragma unroll
            for (int v = 0; v < NV; ++v) {
              const int f4 = lane + v * L;
              if (f4 < NF4 && (lane & (S - 1)) == 0) out[f4 / S] = part[v];
            }
          } else if (lane == 0) {
            const int R = S / L;  // consecutive slots of one segment
            for (int v0 = 0; v0 < NV; v0 += R) {
              float acc = 0.0f;
              for (int v = v0; v < v0 + R && v < NV; ++v) acc += part[v];
              if (v0 * L < NF4) out[(v0 * L) / S] = acc;
            }
          }
        } else {
          float* out = a.out + eid[u] * NF;
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int f4 = lane + v * L;
            if (f4 < NF4)
              st4(out + 4 * f4, make_float4(op1<OP>(l4[u][v].x, r4[u][v].x), op1<OP>(l4[u][v].y, r4[u][v].y),
                                            op1<OP>(l4[u][v].z, r4[u][v].z), op1<OP>(l4[u][v].w, r4[u][v].w)));
          }
        }
      } else {
        const float* go = a.go + pick(a.go_role, row[u], col[u], eid[u]) * a.D;
        float* out = a.out + eid[u] * NF;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int f4 = lane + v * L;
          if (f4 >= NF4) continue;
          float4 g4;
          if (OP == OP_DOT && len > 1) {
            const float ge = go[(4 * f4) / len];
            g4 = make_float4(ge, ge, ge, ge);
          } else {
            g4 = ld4(go + 4 * f4);
          }
          st4(out + 4 * f4, make_float4(bwd1<OP>(g4.x, l4[u][v].x, r4[u][v].x, a.want),
                                        bwd1<OP>(g4.y, l4[u][v].y, r4[u][v].y, a.want),
                                        bwd1<OP>(g4.z, l4[u][v].z, r4[u][v].z, a.want),
                                        bwd1<OP>(g4.w, l4[u][v].w, r4[u][v].w, a.want)));
        }
      }
    }
  }
}

unsigned grid_for(int64_t items, int per_block) {
  // grid-stride: enough blocks to fill 256 CUs several times over
  const int64_t want = (items + per_block - 1) / per_block;
  return static_cast<unsigned>(want < 256 * 64 ? (want > 0 ? want : 1) : 256 * 64);
}

template <int OP, bool BWD>
void run_lane(const SddmmArgs& a, int64_t NF, hipStream_t s) {
  const dim3 grid(grid_for(a.nnz, kBlock)), block(kBlock);
  switch (NF) {
    case 1: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 1>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 2>), grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 3>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 4>), grid, block, 0, s, a); break;
    case 6: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 6>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((k_sddmm_lane<OP, BWD, 8>), grid, block, 0, s, a); break;
  }
}

template <int OP, bool BWD, int L, int NV>
void run_group_cfg(const SddmmArgs& a, hipStream_t s) {
  constexpr int U = GroupUnroll<NV>::U;
  hipLaunchKernelGGL((k_sddmm_group<OP, BWD, L, NV>), dim3(grid_for((a.nnz + U - 1) / U, kBlock / L)),
                     dim3(kBlock), 0, s, a);
}

template <int OP, bool BWD>
void run_group(const SddmmArgs& a, int64_t NF, hipStream_t s) {
  const int64_t NF4 = NF / 4;
  if (NF4 <= 4) run_group_cfg<OP, BWD, 4, 1>(a, s);
  else if (NF4 <= 8) run_group_cfg<OP, BWD, 8, 1>(a, s);
  else if (NF4 <= 16) run_group_cfg<OP, BWD, 16, 1>(a, s);
  else if (NF4 <= 32) run_group_cfg<OP, BWD, 32, 1>(a, s);
  else if (NF4 <= 64) run_group_cfg<OP, BWD, 64, 1>(a, s);
  else if (NF4 <= 128) run_group_cfg<OP, BWD, 64, 2>(a, s);
  else run_group_cfg<OP, BWD, 64, 4>(a, s);
}

int group_lanes(int64_t NF4) {
  int L = 4;
  while (L < NF4 && L < 64) L <<= 1;
  return L;
}

template <bool BWD>
void run_op(int op, const SddmmArgs& a, hipStream_t s) {
  const int64_t NF = a.D * a.len;
  const bool lane = NF <= 8;
#define DGLMI_SDDMM(OPV) \
  if (lane) run_lane<OPV, BWD>(a, NF, s); else run_group<OPV, BWD>(a, NF, s);
  switch (op) {
    case OP_ADD: DGLMI_SDDMM(OP_ADD) break;
    case OP_SUB: DGLMI_SDDMM(OP_SUB) break;
    case OP_MUL: DGLMI_SDDMM(OP_MUL) break;
    case OP_DIV: DGLMI_SDDMM(OP_DIV) break;
    case OP_DOT: DGLMI_SDDMM(OP_DOT) break;
    default: DGLMI_SDDMM(OP_USE_LHS) break;
  }
#undef DGLMI_SDDMM
}

}  // namespace

bool sddmm_supported(int op, bool bwd, int64_t D, int64_t len) {
  const int64_t NF = D * len;
  if (NF <= 0) return false;
  if (NF <= 8) return NF != 5 && NF != 7;
  if (NF % 4 != 0 || NF > 1024) return false;
  if (op == OP_DOT && len > 1) {
    if (len % 4 != 0) return false;
    if (bwd) return true;
    const int64_t S = len / 4;
    if ((S & (S - 1)) != 0) return false;
    const int L = group_lanes(NF / 4);
    if (S > L && S % L != 0) return false;
  }
  return true;
}

void launch_sddmm(int op, bool bwd, const SddmmArgs& a, hipStream_t s) {
  if (a.nnz == 0) return;
  if (bwd) run_op<true>(op, a, s);
  else run_op<false>(op, a, s);
}

}  // namespace dglmi
