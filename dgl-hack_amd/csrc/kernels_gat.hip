// Fused GAT attention + aggregation for gfx950.
//
// The hack's fused GAT (src/kernel/cuda/binary_reduce_impl.cu:46-422 forward,
// :124-357 + 1248-1308 backward; python FusedGat, tensor.py:383-420) replaces
//   u_add_v -> leaky_relu -> edge_softmax -> u_mul_e_sum
// by two kernels that materialise exp[E, H] and sum[N, H] (no max subtraction,
// and an out-of-bounds row loop at :60), and a backward with atomics.
//
// Here, per destination row v and head h, ONE pass over the in-edges computes
//   s_e = leaky(el[u, h] + er[v, h]),  m = max s_e,  l = sum exp(s_e - m),
//   out[v, h, :] = sum exp(s_e - m) / l * ft[u, h, :]
// with an online (running-max) softmax in registers -- no per-edge buffer at
// all; only m and l (N x H) are kept for the backward pass.  Work is cut into
// fixed edge chunks like kernels_spmm.hip; a row split across chunks leaves
// (m, l, acc) partials that the fixup merges with the usual rescaling, in
// chunk order (deterministic).
//
// Backward (attention-backward style, delta = rowsum(grad_out * out)):
//   a_e    = exp(s_e - m_v) / l_v
//   g_e    = <grad_out[v, h, :], ft[u, h, :]>
//   dpre_e = a_e (g_e - delta_v) * (pre_e > 0 ? 1 : slope)
//   grad_er[v] = sum_in dpre   (in-CSR walk, dst-owner; also writes delta and
//                               packed per-(v, h) stats {er, m, 1/l, delta})
//   grad_ft[u] = sum_out a_e grad_out[v],  grad_el[u] = sum_out dpre
//                              (out-CSR walk, src-owner)
// Everything owner-computes: no atomics.
//
// Forward with the slope aggregates (GatArgs::lf / ls, DGLMIFusedGatForwardEx):
// the same pass also keeps, per row and head,
//   ls[v] = sum_in a_e lrelu'(pre_e),   lf[v] = sum_in a_e lrelu'(pre_e) ft[u]
// (lrelu' = 1 or slope, so one more running sum beside out's, rescaled with it), and
//   grad_er[v] = sum_in dpre_e = <grad_out[v], lf[v]> - delta_v ls[v]
// becomes a dense per-row pass (k_gat_stats): the backward needs no in-CSR walk.
#include "internal.h"

#include <climits>
#include <cmath>

namespace dglmi {



namespace {

constexpr int kBlock = 256;
constexpr float kNegInf = -__builtin_huge_valf();

__device__ __forceinline__ float4 ld4g(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4g(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float leaky(float x, float s) { return x > 0.0f ? x : s * x; }
__device__ __forceinline__ float dleaky(float x, float s) { return x > 0.0f ? 1.0f : s; }
// e^x as one v_exp_f32 (2^(x log2 e)): the walks evaluate it once or twice per
// edge and lane, where the accurate expf's range reduction cost ~12 VALU each.
// Relative error ~|x| 2^-24 (< 2e-6 for the logits a softmax sees), far inside
// the 1e-4 budget.  The walks of the forward and the backward both use it; the
// forward's rescales of stored (m, l) partials (the split-row fixup and the
// column-block merge) use the accurate expf, so the attention weights the
// backward recomputes match the forward's within that budget, not bit for bit.
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
// Element offset of (row, off) in a table of rows `w` floats wide: 32-bit
// arithmetic when every offset of the gathered tables fits (GatArgs::o32), one
// v_mul_lo_u32 instead of a 64-bit multiply per gather.
template <bool O32>
__device__ __forceinline__ int64_t roff(int64_t row, int64_t w, int off) {
  if constexpr (O32)
    return static_cast<int64_t>(static_cast<uint32_t>(row) * static_cast<uint32_t>(w) +
                                static_cast<uint32_t>(off));
  else
    return row * w + off;
}
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
// sum over the D4 lanes of one head (D4 = D / 4, a power of two <= L).  Lanes
// 1 and 2 apart swap through DPP quad permutations (no LDS round trip, unlike
// the ds_bpermute of __shfl_xor); wider heads finish with __shfl_xor.  Every
// lane of the head ends with the same sum (a + b == b + a).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float head_sum(float x, int d4) {
  if (d4 >= 2) x += dpp_f<0xB1>(x);  // quad_perm [1, 0, 3, 2]: lane ^ 1
  if (d4 >= 4) x += dpp_f<0x4E>(x);  // quad_perm [2, 3, 0, 1]: lane ^ 2
  for (int off = 4; off < d4; off <<= 1) x += __shfl_xor(x, off);
  return x;
}

// Attention dropout, staged per position: the H <= 32 keep bits of the position's edge
// (one key per edge, one hash per pair of heads), computed by the one lane that stages
// the position instead of by every lane of the head in the edge loop (16 lanes per row
// at 8 x 8).  The edge loop only tests a bit: a hash there (round 4 kept one for
// H > 32, which the compiler evaluated for every edge and selected away) cost ~24 VALU
// instructions per edge and lane.  The C entry takes H <= 32 (gat_set_dropout).
// torch's own draws (drop_rng): the H elements e * H + h of the (E, H) draw, one Philox
// block per run of elements that share a (thread, draw) slot -- two per edge at H = 8
// with vec 4 -- recomputed in every walk instead of a mask read back per edge (DROP 3).
// One 32 x 32 -> 64 multiply as a single v_mad_u64_u32 (hipcc emits v_mul_hi_u32 +
// v_mul_lo_u32): 1.42x the Philox block rate on gfx950 (scripts/philox_rate_probe.hip:
// 657 vs 463 G blocks/s).  The carry-out lands in an SGPR pair, unused.
__device__ __forceinline__ void philox_mul(uint32_t m, uint32_t x, uint32_t& hi, uint32_t& lo) {
  uint64_t r, c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(c) : "v"(m), "v"(x));
  hi = static_cast<uint32_t>(r >> 32);
  lo = static_cast<uint32_t>(r);
}
// two independent Philox4x32-10 blocks in lockstep (the dependent chain of one block is
// latency-bound in the staging lane; two interleave)
__device__ __forceinline__ void philox_pair(Philox4& c0, Philox4& c1, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h00, l00, h01, l01, h10, l10, h11, l11;
    philox_mul(0xD2511F53u, c0.x, h00, l00);
    philox_mul(0xD2511F53u, c1.x, h10, l10);
    philox_mul(0xCD9E8D57u, c0.z, h01, l01);
    philox_mul(0xCD9E8D57u, c1.z, h11, l11);
    c0 = Philox4{h01 ^ c0.y ^ k0, l01, h00 ^ c0.w ^ k1, l00};
    c1 = Philox4{h11 ^ c1.y ^ k0, l11, h10 ^ c1.w ^ k1, l10};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
__device__ __forceinline__ Philox4 draw_counter(const GatArgs& a, const DrawSlot& s) {
  const uint64_t c = a.rng_ctr + static_cast<uint64_t>(s.j);
  const uint64_t t = static_cast<uint64_t>(s.t);
  return Philox4{static_cast<uint32_t>(c), static_cast<uint32_t>(c >> 32), static_cast<uint32_t>(t),
                 static_cast<uint32_t>(t >> 32)};
}
__device__ __forceinline__ uint32_t draw_nibble(const Philox4& r, float keep) {
  return (dropout_draw_kept(r, 0, keep) ? 1u : 0u) | (dropout_draw_kept(r, 1, keep) ? 2u : 0u) |
         (dropout_draw_kept(r, 2, keep) ? 4u : 0u) | (dropout_draw_kept(r, 3, keep) ? 8u : 0u);
}
__device__ __forceinline__ uint32_t gat_draw_keep(const GatArgs& a, int32_t eid) {
  if (a.rng_vec == 4 && (a.H & 3) == 0) {
    // whole blocks: edge e's elements are the uniforms of draws e H / 4 + b, b < H / 4,
    // taken two at a time (H = 8: exactly one pair)
    const uint32_t k0 = static_cast<uint32_t>(a.rng_seed), k1 = static_cast<uint32_t>(a.rng_seed >> 32);
    const int nb = a.H >> 2;
    const int64_t c0 = static_cast<int64_t>(eid) * nb;
    uint32_t kb = 0;
    for (int b = 0; b < nb; b += 2) {
      const int64_t ca = c0 + b, cb = c0 + (b + 1 < nb ? b + 1 : b);
      Philox4 r0 = draw_counter(a, dropout_draw_slot(ca << 2, 4, a.rng_threads, a.rng_shift));
      Philox4 r1 = draw_counter(a, dropout_draw_slot(cb << 2, 4, a.rng_threads, a.rng_shift));
      philox_pair(r0, r1, k0, k1);
      kb |= draw_nibble(r0, a.rng_keep) << (4 * b);
      if (b + 1 < nb) kb |= draw_nibble(r1, a.rng_keep) << (4 * (b + 1));
    }
    return kb;
  }
  uint32_t kb = 0;
  int64_t lt = -1, lj = -1;
  Philox4 r{0u, 0u, 0u, 0u};
  const int64_t i0 = static_cast<int64_t>(eid) * a.H;
  for (int h = 0; h < a.H; ++h) {
    const DrawSlot s = dropout_draw_slot(i0 + h, a.rng_vec, a.rng_threads, a.rng_shift);
    if (s.t != lt || s.j != lj) {
      r = dropout_draw(a.rng_seed, a.rng_ctr, s);
      lt = s.t;
      lj = s.j;
    }
    kb |= (dropout_draw_kept(r, s.comp, a.rng_keep) ? 1u : 0u) << h;
  }
  return kb;
}
__device__ __forceinline__ uint32_t gat_stage_keep(const GatArgs& a, int32_t eid) {
  const uint32_t key = gat_edge_key(a.drop_seed, static_cast<uint32_t>(eid));
  uint32_t kb = 0;
  for (int j = 0; 2 * j < a.H; ++j) {
    const uint32_t r = gat_pair_bits(key, j);
    kb |= ((r & 0xffffu) >= a.drop_thresh ? 1u : 0u) << (2 * j);
    kb |= ((r >> 16) >= a.drop_thresh ? 1u : 0u) << (2 * j + 1);
  }
  return kb;  // bits past H unused
}
__device__ __forceinline__ bool gat_kept(uint32_t staged, int h) { return (staged >> h) & 1u; }
// the caller's keep word of edge e (drop = 2): 8, 16 or 32 bits (a launch-uniform branch)
__device__ __forceinline__ uint32_t gat_keep_word(const GatArgs& a, int32_t e) {
  if (a.drop_width == 8) return static_cast<const uint8_t*>(a.drop_bits)[e];
  if (a.drop_width == 16) return static_cast<const uint16_t*>(a.drop_bits)[e];
  return static_cast<const uint32_t*>(a.drop_bits)[e];
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// LS: also the slope aggregates lf / ls (carry record [acc F][m H][l H][lf F][ls H])
// DROP: attention dropout (a separate instance, so the plain walk's code is untouched):
// 1 the hashed mask, 2 the caller's keep words (GatArgs.drop_bits), 3 torch's dropout
// draws recomputed from the generator state (GatArgs.drop_rng)
template <int L, int NV, bool O32, bool LS, int DROP = 0>
__global__ void __launch_bounds__(kBlock) k_gat_fwd(GatArgs a) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront");
  constexpr int G = kBlock / L;
  constexpr int B = L > 16 ? L : 16;
  constexpr int U = NV == 1 ? 8 : 4;
  __shared__ int32_t s_row[G][B];
  __shared__ int32_t s_col[G][B];
  __shared__ uint32_t s_keep[DROP ? G : 1][DROP ? B : 1];  // dropout keep bits (gat_stage_keep)
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // the fixup's counters
  const int F4 = static_cast<int>(a.F / 4);
  const int H = a.H, D = a.D;
  const int64_t CW = LS ? 2 * a.F + 3 * H : a.F + 2 * H;  // carry record, see above
  constexpr bool drop = DROP != 0;
  constexpr bool table = DROP == 2;  // the caller's keep words, else the hash
  constexpr bool draw = DROP == 3;   // torch's dropout draws (gat_draw_keep)
  int hd[NV], fl[NV];
  bool ok4[NV], lead[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    ok4[v] = f4 < F4;
    fl[v] = 4 * (ok4[v] ? f4 : F4 - 1);  // gathers of idle slots re-read the last one
    hd[v] = ok4[v] ? (4 * f4) / D : 0;
    lead[v] = ok4[v] && ((4 * f4) % D == 0);
  }
  const float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
  auto zero_row = [&](int64_t r) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (ok4[v]) st4g(a.out + r * a.F + 4 * (lane + v * L), Z);
      if (LS && ok4[v]) st4g(a.lf + r * a.F + 4 * (lane + v * L), Z);
      if (lead[v]) {
        a.m[r * H + hd[v]] = 0.0f;
        a.l[r * H + hd[v]] = 0.0f;
        if (LS) a.ls[r * H + hd[v]] = 0.0f;
      }
    }
  };
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  float mx[NV], sm[NV], erv[NV], qs[NV];
  float4 acc[NV], qa[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    mx[v] = kNegInf;
    sm[v] = 0.0f;
    acc[v] = Z;
    qs[v] = 0.0f;
    qa[v] = Z;
    erv[v] = ok4[v] ? a.er[cur * H + hd[v]] : 0.0f;
  }
  // write a finished / partial row.  final: normalise; else raw (m, l, acc)
  auto flush = [&](int64_t r, bool is_cont, bool final) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (!ok4[v]) continue;
      const int f4 = lane + v * L;
      if (is_cont) {
        float* c = a.carry + chunk * CW;
        st4g(c + 4 * f4, acc[v]);
        if (LS) st4g(c + a.F + 2 * H + 4 * f4, qa[v]);
        if (lead[v]) {
          c[a.F + hd[v]] = mx[v];
          c[a.F + H + hd[v]] = sm[v];
          if (LS) c[2 * a.F + 2 * H + hd[v]] = qs[v];
        }
      } else {
        float4 o = acc[v], q = qa[v];
        float qsv = qs[v];
        if (final && !a.raw) {
          const float inv = sm[v] > 0.0f ? 1.0f / sm[v] : 0.0f;
          o = make_float4(o.x * inv, o.y * inv, o.z * inv, o.w * inv);
          q = make_float4(q.x * inv, q.y * inv, q.z * inv, q.w * inv);
          qsv *= inv;
        }
        st4g(a.out + r * a.F + 4 * f4, o);
        if (LS) st4g(a.lf + r * a.F + 4 * f4, q);
        if (lead[v]) {
          a.m[r * H + hd[v]] = mx[v];
          a.l[r * H + hd[v]] = sm[v];
          if (LS) a.ls[r * H + hd[v]] = qsv;
        }
      }
    }
  };
  // the batch's row / column (and, with dropout, edge) ids are loaded one batch ahead,
  // into registers, while this batch's gathers are in flight (round 5): the staging
  // loads, and the edge-id load the keep-bit hash waits for, are off the critical path
  constexpr int SQ = B / L;  // positions each lane stages per batch
  int32_t nr[SQ], nc[SQ], ne[drop ? SQ : 1];
  uint32_t nk[table ? SQ : 1];
  // caller's mask (DROP 2): a batch's keep words are loaded with its row / column ids,
  // from edge ids loaded one batch earlier still, so the dependent load never waits
  auto fetch = [&](int64_t nb) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int64_t p = nb + lane + i * L;
      const bool ok = p < p1;
      nr[i] = ok ? a.rows[p] : INT_MAX;
      nc[i] = ok ? a.indices[p] : 0;
      if constexpr (table) {
        if (a.drop_pos) {  // position order: one coalesced byte / word per position
          nk[table ? i : 0] = ok ? gat_keep_word(a, static_cast<int32_t>(a.drop_off + p)) : 0u;
        } else {
          nk[table ? i : 0] = ok ? gat_keep_word(a, ne[table ? i : 0]) : 0u;
          ne[table ? i : 0] = p + B < p1 ? a.eids[p + B] : 0;
        }
      } else if constexpr (drop) {
        ne[drop ? i : 0] = ok ? a.eids[p] : 0;
      }
    }
  };
  if constexpr (table) {
    if (!a.drop_pos) {
#pragma unroll
      for (int i = 0; i < SQ; ++i) {
        const int64_t p = p0 + lane + i * L;
        ne[table ? i : 0] = p < p1 ? a.eids[p] : 0;
      }
    }
  }
  fetch(p0);
  for (int64_t base = p0; base < p1; base += B) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int q = lane + i * L;
      s_row[g][q] = nr[i];
      s_col[g][q] = nc[i];
      if constexpr (drop)
        s_keep[drop ? g : 0][drop ? q : 0] =
            nr[i] == INT_MAX ? 0u
            : table ? nk[table ? i : 0]
            : draw  ? gat_draw_keep(a, ne[drop ? i : 0])
                    : gat_stage_keep(a, ne[drop ? i : 0]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (base + B < p1) fetch(base + B);
#pragma unroll
    for (int ub = 0; ub < B; ub += U) {
      float4 val[U][NV];
      float elv[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // unconditional: positions past the chunk carry column 0 (a valid row),
        // and the loop below stops at them
        const int64_t col = s_col[g][ub + u];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          val[u][v] = ld4g(a.ft + roff<O32>(col, a.F, fl[v]));
          elv[u][v] = a.el[roff<O32>(col, H, hd[v])];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t r = s_row[g][ub + u];
        if (r == INT_MAX) break;
        if (r != cur) {
          flush(cur, cont, true);
          cur = r;
          cont = false;
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            mx[v] = kNegInf;
            sm[v] = 0.0f;
            acc[v] = Z;
            qs[v] = 0.0f;
            qa[v] = Z;
            erv[v] = ok4[v] ? a.er[cur * H + hd[v]] : 0.0f;
          }
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const float pre = elv[u][v] + erv[v];
          const float s = leaky(pre, a.slope);
          if (s > mx[v]) {
            const float sc = fexp(mx[v] - s);
            acc[v] = make_float4(acc[v].x * sc, acc[v].y * sc, acc[v].z * sc, acc[v].w * sc);
            sm[v] *= sc;
            if (LS) {
              qa[v] = make_float4(qa[v].x * sc, qa[v].y * sc, qa[v].z * sc, qa[v].w * sc);
              qs[v] *= sc;
            }
            mx[v] = s;
          }
          const float pe = fexp(s - mx[v]);
          // dropout: the output and lf take the kept, rescaled weight; the softmax
          // denominator and ls the plain one
          float pk = pe;
          if constexpr (drop)
            pk = gat_kept(s_keep[drop ? g : 0][drop ? ub + u : 0], hd[v]) ? pe * a.drop_scale : 0.0f;
          const float4 x = val[u][v];
          acc[v] = make_float4(acc[v].x + pk * x.x, acc[v].y + pk * x.y, acc[v].z + pk * x.z,
                               acc[v].w + pk * x.w);
          sm[v] += pe;
          if (LS) {
            const float dl = dleaky(pre, a.slope);
            const float pd = pk * dl;
            qa[v] = make_float4(qa[v].x + pd * x.x, qa[v].y + pd * x.y, qa[v].z + pd * x.z,
                                qa[v].w + pd * x.w);
            qs[v] += pe * dl;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  const bool continues = p1 < a.nnz && a.rows[p1] == cur;
  flush(cur, cont, !continues);
  fill_empty_rows(a.indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, L, lane, zero_row);
}

template <int L, int NV, bool LS>
__global__ void __launch_bounds__(kBlock) k_gat_fwd_fixup(GatArgs a) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront");
  constexpr int G = kBlock / L;
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
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
  const int64_t cend = nseg == 1 ? last : (chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last);
  const int F4 = static_cast<int>(a.F / 4);
  const int H = a.H;
  const int64_t CW = LS ? 2 * a.F + 3 * H : a.F + 2 * H;
  // online-softmax merge of carry record c into (acc, mx, sm) (and the slope
  // aggregates (qa, qs), rescaled by the same factors)
  auto merge = [&](float4& acc, float& mx, float& sm, float4& qa, float& qs, int64_t c, int f4,
                   int h) {
    const float* cr = a.carry + c * CW;
    const float4 ca = ld4g(cr + 4 * f4);
    const float cm = cr[a.F + h], cl = cr[a.F + H + h];
    const float mn = fmaxf(mx, cm);
    const float f1 = expf(mx - mn), f2 = expf(cm - mn);
    acc = make_float4(acc.x * f1 + ca.x * f2, acc.y * f1 + ca.y * f2, acc.z * f1 + ca.z * f2,
                      acc.w * f1 + ca.w * f2);
    sm = sm * f1 + cl * f2;
    if (LS) {
      const float4 cq = ld4g(cr + a.F + 2 * H + 4 * f4);
      qa = make_float4(qa.x * f1 + cq.x * f2, qa.y * f1 + cq.y * f2, qa.z * f1 + cq.z * f2,
                       qa.w * f1 + cq.w * f2);
      qs = qs * f1 + cr[2 * a.F + 2 * H + h] * f2;
    }
    mx = mn;
  };
  if (nseg > 1) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      if (f4 >= F4) continue;
      const int h = (4 * f4) / a.D;
      float* cr = a.carry + chunk * CW;
      float4 acc = ld4g(cr + 4 * f4);
      float mx = cr[a.F + h], sm = cr[a.F + H + h];
      float4 qa = LS ? ld4g(cr + a.F + 2 * H + 4 * f4) : make_float4(0.f, 0.f, 0.f, 0.f);
      float qs = LS ? cr[2 * a.F + 2 * H + h] : 0.0f;
      for (int64_t c = chunk + 1; c <= cend; ++c) merge(acc, mx, sm, qa, qs, c, f4, h);
      st4g(cr + 4 * f4, acc);
      if (LS) st4g(cr + a.F + 2 * H + 4 * f4, qa);
      if ((4 * f4) % a.D == 0) {
        cr[a.F + h] = mx;
        cr[a.F + H + h] = sm;
        if (LS) cr[2 * a.F + 2 * H + h] = qs;
      }
    }
    if (!seg_arrive_last(a.seg_cnt + first, nseg, L, lane)) return;
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    if (f4 >= F4) continue;
    const int h = (4 * f4) / a.D;
    float4 acc = ld4g(a.out + r * a.F + 4 * f4);
    float mx = a.m[r * H + h], sm = a.l[r * H + h];
    float4 qa = LS ? ld4g(a.lf + r * a.F + 4 * f4) : make_float4(0.f, 0.f, 0.f, 0.f);
    float qs = LS ? a.ls[r * H + h] : 0.0f;
    if (nseg > 1)
      for (int64_t sg = 0; sg < nseg; ++sg) merge(acc, mx, sm, qa, qs, first + sg * kFixSeg, f4, h);
    else
      for (int64_t c = first; c <= last; ++c) merge(acc, mx, sm, qa, qs, c, f4, h);
    const float inv = a.raw ? 1.0f : (sm > 0.0f ? 1.0f / sm : 0.0f);
    st4g(a.out + r * a.F + 4 * f4, make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
    if (LS) st4g(a.lf + r * a.F + 4 * f4, make_float4(qa.x * inv, qa.y * inv, qa.z * inv, qa.w * inv));
    if ((4 * f4) % a.D == 0) {
      a.m[r * H + h] = mx;
      a.l[r * H + h] = sm;
      if (LS) a.ls[r * H + h] = qs * inv;
    }
  }
}

// ---------------------------------------------------------------------------
// backward, destination side (in-CSR): grad_er, delta, packed stats
// DROP 3: torch's dropout draws (the backward of a forward without slope aggregates:
// GATConv's composition, backend.GatComposition): an edge's attention gradient term takes
// its kept, rescaled <grad_out, ft>; delta = <grad_out, out> is the dropped output's.
// ---------------------------------------------------------------------------
template <int L, int NV, bool O32, int DROP = 0>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_dst(GatArgs a) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront");
  static_assert(DROP == 0 || DROP == 3, "the destination walk takes only the recomputed draws");
  constexpr int G = kBlock / L;
  constexpr int B = L > 16 ? L : 16;
  constexpr int U = NV == 1 ? 8 : 4;
  __shared__ int32_t s_row[G][B];
  __shared__ int32_t s_col[G][B];
  __shared__ uint32_t s_keep[DROP ? G : 1][DROP ? B : 1];
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // the fixup's counters
  const int F4 = static_cast<int>(a.F / 4);
  const int H = a.H, D = a.D, D4 = a.D / 4;
  int hd[NV], fl[NV];
  bool ok4[NV], lead[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    ok4[v] = f4 < F4;
    fl[v] = 4 * (ok4[v] ? f4 : F4 - 1);  // gathers of idle slots re-read the last one
    hd[v] = ok4[v] ? (4 * f4) / D : 0;
    lead[v] = ok4[v] && ((4 * f4) % D == 0);
  }
  const float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 gov[NV];
  float erv[NV], mv[NV], linv[NV], dlt[NV], acc[NV];
  // per-row state: grad_out slice, er, m, 1/l, delta = <grad_out, out> per head
  auto load_row = [&](int64_t r) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      gov[v] = ok4[v] ? ld4g(a.go + r * a.F + 4 * f4) : Z;
      const float4 fo = ok4[v] ? ld4g(a.fo + r * a.F + 4 * f4) : Z;
      dlt[v] = head_sum(dot4(gov[v], fo), D4);
      erv[v] = ok4[v] ? a.er[r * H + hd[v]] : 0.0f;
      mv[v] = ok4[v] ? a.m_in[r * H + hd[v]] : 0.0f;
      const float lv = ok4[v] ? a.l_in[r * H + hd[v]] : 0.0f;
      linv[v] = lv > 0.0f ? 1.0f / lv : 0.0f;
      acc[v] = 0.0f;
    }
  };
  auto flush = [&](int64_t r, bool is_cont) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (!lead[v]) continue;
      if (is_cont) {
        a.carry[chunk * H + hd[v]] = acc[v];
      } else {
        float* ge = a.g_er + r * H + hd[v];
        *ge = a.accumulate ? *ge + acc[v] : acc[v];
        if (!a.skip_stats) a.stats[r * H + hd[v]] = make_float4(erv[v], mv[v], linv[v], dlt[v]);
      }
    }
  };
  // a row without edges (in this launch): no gradient; its stats are the row's own
  // forward values (m = l = 0 and delta = 0 for a row without any in-edge), so the
  // source-side walk of a column-blocked backward reads them for every row
  auto zero_row = [&](int64_t r) {
    if (!a.skip_stats) {
      load_row(r);
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if (lead[v]) a.stats[r * H + hd[v]] = make_float4(erv[v], mv[v], linv[v], dlt[v]);
    }
    if (!a.accumulate) {
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if (lead[v]) a.g_er[r * H + hd[v]] = 0.0f;
    }
  };
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  load_row(cur);
  for (int64_t base = p0; base < p1; base += B) {
    for (int q = lane; q < B; q += L) {
      const int64_t p = base + q;
      const bool ok = p < p1;
      s_row[g][q] = ok ? a.rows[p] : INT_MAX;
      s_col[g][q] = ok ? a.indices[p] : 0;
      if constexpr (DROP == 3) s_keep[DROP ? g : 0][DROP ? q : 0] = ok ? gat_draw_keep(a, a.eids[p]) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int ub = 0; ub < B; ub += U) {
      float4 ftv[U][NV];
      float elv[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t col = s_col[g][ub + u];  // 0 (a valid row) past the chunk
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          ftv[u][v] = ld4g(a.ft + roff<O32>(col, a.F, fl[v]));
          elv[u][v] = a.el[roff<O32>(col, H, hd[v])];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t r = s_row[g][ub + u];
        if (r == INT_MAX) break;
        if (r != cur) {
          flush(cur, cont);
          cur = r;
          cont = false;
          load_row(cur);
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const float pre = elv[u][v] + erv[v];
          const float att = fexp(leaky(pre, a.slope) - mv[v]) * linv[v];
          float ge = head_sum(dot4(gov[v], ftv[u][v]), D4);
          if constexpr (DROP == 3)
            ge = gat_kept(s_keep[DROP ? g : 0][DROP ? ub + u : 0], hd[v]) ? ge * a.drop_scale : 0.0f;
          acc[v] += att * (ge - dlt[v]) * dleaky(pre, a.slope);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  flush(cur, cont);
  fill_empty_rows(a.indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, L, lane, zero_row);
}

// ---------------------------------------------------------------------------
// backward, source side (out-CSR): grad_ft, grad_el
// ---------------------------------------------------------------------------
template <int L, int NV, bool O32, int DROP>
__device__ __forceinline__ void gat_bwd_src_body(const GatArgs& a) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront");
  constexpr int G = kBlock / L;
  constexpr int B = L > 16 ? L : 16;
  constexpr int U = NV == 1 ? 8 : 4;
  __shared__ int32_t s_row[G][B];
  __shared__ int32_t s_col[G][B];
  __shared__ uint32_t s_keep[DROP ? G : 1][DROP ? B : 1];  // dropout keep bits (gat_stage_keep)
  constexpr bool drop = DROP != 0;
  constexpr bool table = DROP == 2;  // the caller's keep words, else the hash
  constexpr bool draw = DROP == 3;   // torch's dropout draws (gat_draw_keep)
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
  const int64_t K = a.chunk;
  const int64_t p0 = chunk * K;
  if (p0 >= a.nnz) return;
  const int64_t p1 = p0 + K < a.nnz ? p0 + K : a.nnz;
  if (a.seg_cnt != nullptr && lane == 0) a.seg_cnt[chunk] = 0;  // the fixup's counters
  const int F4 = static_cast<int>(a.F / 4);
  const int H = a.H, D = a.D, D4 = a.D / 4;
  const int64_t CW = a.F + H;
  int hd[NV], fl[NV];
  bool ok4[NV], lead[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    ok4[v] = f4 < F4;
    fl[v] = 4 * (ok4[v] ? f4 : F4 - 1);  // gathers of idle slots re-read the last one
    hd[v] = ok4[v] ? (4 * f4) / D : 0;
    lead[v] = ok4[v] && ((4 * f4) % D == 0);
  }
  const float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
  auto zero_row = [&](int64_t r) {
    if (a.accumulate) return;  // nothing to add
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (ok4[v]) st4g(a.g_ft + r * a.F + 4 * (lane + v * L), Z);
      if (lead[v]) a.g_el[r * H + hd[v]] = 0.0f;
    }
  };
  float4 ftv[NV], accf[NV];
  float elv[NV], acce[NV];
  auto load_row = [&](int64_t r) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      ftv[v] = ok4[v] ? ld4g(a.ft + r * a.F + 4 * f4) : Z;
      elv[v] = ok4[v] ? a.el[r * H + hd[v]] : 0.0f;
      accf[v] = Z;
      acce[v] = 0.0f;
    }
  };
  auto flush = [&](int64_t r, bool is_cont) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (!ok4[v]) continue;
      const int f4 = lane + v * L;
      float* dst = is_cont ? a.carry + chunk * CW : a.g_ft + r * a.F;
      float4 val = accf[v];
      if (!is_cont && a.accumulate) {
        const float4 o = ld4g(dst + 4 * f4);
        val = make_float4(o.x + val.x, o.y + val.y, o.z + val.z, o.w + val.w);
      }
      st4g(dst + 4 * f4, val);
      if (lead[v]) {
        if (is_cont) a.carry[chunk * CW + a.F + hd[v]] = acce[v];
        else if (a.accumulate) a.g_el[r * H + hd[v]] += acce[v];
        else a.g_el[r * H + hd[v]] = acce[v];
      }
    }
  };
  int64_t cur = a.rows[p0];
  bool cont = p0 > 0 && a.rows[p0 - 1] == cur;
  load_row(cur);
  // the batch's row / column (and, with dropout, edge) ids are loaded one batch ahead,
  // into registers, while this batch's gathers are in flight (round 5): the staging
  // loads, and the edge-id load the keep-bit hash waits for, are off the critical path
  constexpr int SQ = B / L;  // positions each lane stages per batch
  int32_t nr[SQ], nc[SQ], ne[drop ? SQ : 1];
  uint32_t nk[table ? SQ : 1];
  // caller's mask (DROP 2): a batch's keep words are loaded with its row / column ids,
  // from edge ids loaded one batch earlier still, so the dependent load never waits
  auto fetch = [&](int64_t nb) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int64_t p = nb + lane + i * L;
      const bool ok = p < p1;
      nr[i] = ok ? a.rows[p] : INT_MAX;
      nc[i] = ok ? a.indices[p] : 0;
      if constexpr (table) {
        if (a.drop_pos) {  // position order: one coalesced byte / word per position
          nk[table ? i : 0] = ok ? gat_keep_word(a, static_cast<int32_t>(a.drop_off + p)) : 0u;
        } else {
          nk[table ? i : 0] = ok ? gat_keep_word(a, ne[table ? i : 0]) : 0u;
          ne[table ? i : 0] = p + B < p1 ? a.eids[p + B] : 0;
        }
      } else if constexpr (drop) {
        ne[drop ? i : 0] = ok ? a.eids[p] : 0;
      }
    }
  };
  if constexpr (table) {
    if (!a.drop_pos) {
#pragma unroll
      for (int i = 0; i < SQ; ++i) {
        const int64_t p = p0 + lane + i * L;
        ne[table ? i : 0] = p < p1 ? a.eids[p] : 0;
      }
    }
  }
  fetch(p0);
  for (int64_t base = p0; base < p1; base += B) {
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      const int q = lane + i * L;
      s_row[g][q] = nr[i];
      s_col[g][q] = nc[i];
      if constexpr (drop)
        s_keep[drop ? g : 0][drop ? q : 0] =
            nr[i] == INT_MAX ? 0u
            : table ? nk[table ? i : 0]
            : draw  ? gat_draw_keep(a, ne[drop ? i : 0])
                    : gat_stage_keep(a, ne[drop ? i : 0]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (base + B < p1) fetch(base + B);
#pragma unroll
    for (int ub = 0; ub < B; ub += U) {
      float4 gov[U][NV], st[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t col = s_col[g][ub + u];  // 0 (a valid row) past the chunk
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          gov[u][v] = ld4g(a.go + roff<O32>(col, a.F, fl[v]));
          st[u][v] = a.stats[roff<O32>(col, H, hd[v])];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t r = s_row[g][ub + u];
        if (r == INT_MAX) break;
        if (r != cur) {
          flush(cur, cont);
          cur = r;
          cont = false;
          load_row(cur);
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const float4 sv = st[u][v];  // {er, m, 1/l, delta} of the destination
          const float pre = elv[v] + sv.x;
          const float att = fexp(leaky(pre, a.slope) - sv.y) * sv.z;
          const float4 gv = gov[u][v];
          const float ge = head_sum(dot4(gv, ftv[v]), D4);
          // dropout: d = kept ? 1 / (1 - p) : 0 scales the edge's message, not the
          // softmax (grad of the logit: att (d <grad_out, ft> - delta) lrelu')
          float dk = 1.0f;
          if constexpr (drop)
            dk = gat_kept(s_keep[drop ? g : 0][drop ? ub + u : 0], hd[v]) ? a.drop_scale : 0.0f;
          const float te = att * (dk * ge - sv.w) * dleaky(pre, a.slope);
          acce[v] += te;
          // the edge's grad_er term, in this walk's position order (edge-position
          // backward: grad_er is then one gather-sum over the in-CSR)
          if (a.t != nullptr && lead[v]) a.t[(a.t_off + base + ub + u) * H + hd[v]] = te;
          const float ad = att * dk;
          accf[v] = make_float4(accf[v].x + ad * gv.x, accf[v].y + ad * gv.y,
                                accf[v].z + ad * gv.z, accf[v].w + ad * gv.w);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  flush(cur, cont);
  fill_empty_rows(a.indptr, a.num_rows, chunk, (a.nnz + K - 1) / K, L, lane, zero_row);
}

template <int L, int NV, bool O32, int DROP = 0>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_src(GatArgs a) {
  gat_bwd_src_body<L, NV, O32, DROP>(a);
}
// (The dropout instance takes 129 VGPRs and three waves per SIMD; held to four by
// amdgpu_waves_per_eu(4) it spilled two registers and ran no faster: 632 vs 627 us per
// C3 block launch, profiles/r05_c3_and_dropout.json.)

// carries of the backward walks: plain sums (W floats per chunk record, the first
// `wf` of them are per-float4 slots, the rest per head)
template <int L, int NV>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_fixup(GatArgs a, float* vec_out, float* head_out,
                                                          int with_vec) {
  static_assert(L >= 1 && L <= 64, "a lane group must fit in one wavefront");
  constexpr int G = kBlock / L;
  const int g = threadIdx.x / L;
  const int lane = threadIdx.x % L;
  const int64_t chunk = (int64_t)blockIdx.x * G + g;
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
  const int64_t cend = nseg == 1 ? last : (chunk + kFixSeg - 1 < last ? chunk + kFixSeg - 1 : last);
  const int F4 = static_cast<int>(a.F / 4);
  const int H = a.H;
  const int64_t CW = with_vec ? a.F + H : H;
  const int64_t hoff = with_vec ? a.F : 0;
  const float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](float4& accf, float& acce, int64_t c, int f4, int h, bool lead) {
    const float* cr = a.carry + c * CW;
    if (with_vec) {
      const float4 t = ld4g(cr + 4 * f4);
      accf = make_float4(accf.x + t.x, accf.y + t.y, accf.z + t.z, accf.w + t.w);
    }
    if (lead) acce += cr[hoff + h];
  };
  if (nseg > 1) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int f4 = lane + v * L;
      if (f4 >= F4) continue;
      const int h = (4 * f4) / a.D;
      const bool lead = (4 * f4) % a.D == 0;
      float4 accf = Z;
      float acce = 0.0f;
      for (int64_t c = chunk; c <= cend; ++c) add(accf, acce, c, f4, h, lead);
      float* cr = a.carry + chunk * CW;
      if (with_vec) st4g(cr + 4 * f4, accf);
      if (lead) cr[hoff + h] = acce;
    }
    if (!seg_arrive_last(a.seg_cnt + first, nseg, L, lane)) return;
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f4 = lane + v * L;
    if (f4 >= F4) continue;
    const int h = (4 * f4) / a.D;
    const bool lead = (4 * f4) % a.D == 0;
    float4 accf = with_vec ? ld4g(vec_out + r * a.F + 4 * f4) : Z;
    float acce = lead ? head_out[r * H + h] : 0.0f;
    if (nseg > 1)
      for (int64_t sg = 0; sg < nseg; ++sg) add(accf, acce, first + sg * kFixSeg, f4, h, lead);
    else
      for (int64_t c = first; c <= last; ++c) add(accf, acce, c, f4, h, lead);
    if (with_vec) st4g(vec_out + r * a.F + 4 * f4, accf);
    if (lead) head_out[r * H + h] = acce;
  }
}

// Merge the unnormalised per-block softmax partials of a column-blocked forward
// (blocks in order; a block that saw no edge of the row has l = 0 and is skipped).
// lf_part / ls_part (may be NULL): the blocks' raw slope aggregates, merged into lf / ls
// with the same factors.
__global__ void __launch_bounds__(kBlock) k_gat_merge(const float* __restrict__ out_part,
                                                     const float* __restrict__ m_part,
                                                     const float* __restrict__ l_part, int nb,
                                                     int64_t num_rows, int H, int D,
                                                     float* __restrict__ out, float* __restrict__ m,
                                                     float* __restrict__ l,
                                                     const float* __restrict__ lf_part,
                                                     const float* __restrict__ ls_part,
                                                     float* __restrict__ lf, float* __restrict__ ls) {
  const int64_t F = static_cast<int64_t>(H) * D;
  const int64_t F4 = F / 4;
  const int64_t total = num_rows * F4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / F4;
    const int f4 = static_cast<int>(i - r * F4);
    const int h = (4 * f4) / D;
    float mx = kNegInf, sm = 0.0f, qs = 0.0f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f), qa = acc;
    for (int b = 0; b < nb; ++b) {
      const int64_t hi = (static_cast<int64_t>(b) * num_rows + r) * H + h;
      const float lb = l_part[hi];
      if (!(lb > 0.0f)) continue;
      const float mb = m_part[hi];
      const int64_t vi = (static_cast<int64_t>(b) * num_rows + r) * F + 4 * f4;
      const float4 ab = ld4g(out_part + vi);
      const float mn = fmaxf(mx, mb);
      const float f1 = expf(mx - mn), f2 = expf(mb - mn);
      acc = make_float4(acc.x * f1 + ab.x * f2, acc.y * f1 + ab.y * f2, acc.z * f1 + ab.z * f2,
                        acc.w * f1 + ab.w * f2);
      sm = sm * f1 + lb * f2;
      if (lf_part != nullptr) {
        const float4 qb = ld4g(lf_part + vi);
        qa = make_float4(qa.x * f1 + qb.x * f2, qa.y * f1 + qb.y * f2, qa.z * f1 + qb.z * f2,
                         qa.w * f1 + qb.w * f2);
        qs = qs * f1 + ls_part[hi] * f2;
      }
      mx = mn;
    }
    const float inv = sm > 0.0f ? 1.0f / sm : 0.0f;
    st4g(out + r * F + 4 * f4, make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
    if (lf_part != nullptr)
      st4g(lf + r * F + 4 * f4, make_float4(qa.x * inv, qa.y * inv, qa.z * inv, qa.w * inv));
    if ((4 * f4) % D == 0) {
      m[r * H + h] = sm > 0.0f ? mx : 0.0f;
      l[r * H + h] = sm;
      if (lf_part != nullptr) ls[r * H + h] = qs * inv;
    }
  }
}

// Destination stats without a destination-side walk (edge-position backward, and the
// backward after a forward with slope aggregates, which also gets grad_er here): one
// thread per float4 slot of a row, the head's D4 slots adjacent and aligned in the
// wavefront, so delta is reduced by the same head_sum as the destination walk's
// (bit-identical stats).  Every lane reaches the shuffles (no early exit).
__global__ void k_gat_stats(GatArgs a) {
  const int F4 = static_cast<int>(a.F / 4), D4 = a.D / 4;
  const int64_t n = a.num_rows * F4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t start = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t span = (n + stride - 1) / stride * stride;  // wave-uniform trip count
  for (int64_t i = start; i < span; i += stride) {
    const bool ok = i < n;
    const int64_t r = ok ? i / F4 : 0;
    const int f4 = ok ? static_cast<int>(i - r * F4) : 0;
    const float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g = ok ? ld4g(a.go + r * a.F + 4 * f4) : Z;
    const float4 o = ok ? ld4g(a.fo + r * a.F + 4 * f4) : Z;
    const float d = head_sum(dot4(g, o), D4);
    // with the forward's slope aggregates: grad_er = <grad_out, lf> - delta ls (no walk)
    const float4 q = (a.lf != nullptr && ok) ? ld4g(a.lf + r * a.F + 4 * f4) : Z;
    const float e = a.lf != nullptr ? head_sum(dot4(g, q), D4) : 0.0f;
    if (ok && f4 % D4 == 0) {
      const int64_t j = r * a.H + f4 / D4;
      const float l = a.l_in[j];
      a.stats[j] = make_float4(a.er[j], a.m_in[j], l > 0.0f ? 1.0f / l : 0.0f, d);
      if (a.lf != nullptr) a.g_er[j] = e - d * a.ls[j];
    }
  }
}

struct Cfg {
  int L, NV;
};
Cfg pick(int64_t F) {
  const int64_t F4 = F / 4;
  if (F4 <= 4) return {4, 1};
  if (F4 <= 8) return {8, 1};
  if (F4 <= 16) return {16, 1};
  if (F4 <= 32) return {32, 1};
  if (F4 <= 64) return {64, 1};
  if (F4 <= 128) return {64, 2};
  return {64, 4};
}

template <int L, int NV>
void fwd_cfg(const GatArgs& a, hipStream_t s) {
  constexpr int G = kBlock / L;
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = static_cast<unsigned>((chunks + G - 1) / G);
  const bool ls = a.lf != nullptr;
#define DGLMI_GAT_FWD(O_, LS_) \
  hipLaunchKernelGGL((k_gat_fwd<L, NV, O_, LS_>), dim3(blocks), dim3(kBlock), 0, s, a)
  if (a.drop == 2) {  // dropout instances for 32-bit offsets only (checked by the C entry)
    if (ls) hipLaunchKernelGGL((k_gat_fwd<L, NV, true, true, 2>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_gat_fwd<L, NV, true, false, 2>), dim3(blocks), dim3(kBlock), 0, s, a);
  } else if (a.drop && a.drop_rng) {
    if (ls) hipLaunchKernelGGL((k_gat_fwd<L, NV, true, true, 3>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_gat_fwd<L, NV, true, false, 3>), dim3(blocks), dim3(kBlock), 0, s, a);
  } else if (a.drop) {
    if (ls) hipLaunchKernelGGL((k_gat_fwd<L, NV, true, true, 1>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_gat_fwd<L, NV, true, false, 1>), dim3(blocks), dim3(kBlock), 0, s, a);
  } else if (a.o32) {
    if (ls) DGLMI_GAT_FWD(true, true); else DGLMI_GAT_FWD(true, false);
  } else {
    if (ls) DGLMI_GAT_FWD(false, true); else DGLMI_GAT_FWD(false, false);
  }
#undef DGLMI_GAT_FWD
  if (chunks > 1) {
    if (ls) hipLaunchKernelGGL((k_gat_fwd_fixup<L, NV, true>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_gat_fwd_fixup<L, NV, false>), dim3(blocks), dim3(kBlock), 0, s, a);
  }
}

template <int L, int NV>
void bwd_dst_cfg(const GatArgs& a, hipStream_t s) {
  constexpr int G = kBlock / L;
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = static_cast<unsigned>((chunks + G - 1) / G);
  if (a.drop)  // the recomputed draws only, 32-bit offsets (checked by the C entry)
    hipLaunchKernelGGL((k_gat_bwd_dst<L, NV, true, 3>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (a.o32)
    hipLaunchKernelGGL((k_gat_bwd_dst<L, NV, true>), dim3(blocks), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((k_gat_bwd_dst<L, NV, false>), dim3(blocks), dim3(kBlock), 0, s, a);
  if (chunks > 1)
    hipLaunchKernelGGL((k_gat_bwd_fixup<L, NV>), dim3(blocks), dim3(kBlock), 0, s, a,
                       static_cast<float*>(nullptr), a.g_er, 0);
}

template <int L, int NV>
void bwd_src_cfg(const GatArgs& a, hipStream_t s) {
  constexpr int G = kBlock / L;
  const int64_t chunks = (a.nnz + a.chunk - 1) / a.chunk;
  const unsigned blocks = static_cast<unsigned>((chunks + G - 1) / G);
  if (a.drop == 2)  // dropout instances for 32-bit offsets only (checked by the C entry)
    hipLaunchKernelGGL((k_gat_bwd_src<L, NV, true, 2>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (a.drop && a.drop_rng)
    hipLaunchKernelGGL((k_gat_bwd_src<L, NV, true, 3>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (a.drop)
    hipLaunchKernelGGL((k_gat_bwd_src<L, NV, true, 1>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (a.o32)
    hipLaunchKernelGGL((k_gat_bwd_src<L, NV, true>), dim3(blocks), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((k_gat_bwd_src<L, NV, false>), dim3(blocks), dim3(kBlock), 0, s, a);
  if (chunks > 1)
    hipLaunchKernelGGL((k_gat_bwd_fixup<L, NV>), dim3(blocks), dim3(kBlock), 0, s, a, a.g_ft,
                       a.g_el, 1);
}

#define DGLMI_GAT_DISPATCH(FN, a, s)                   \
  do {                                                 \
    const Cfg c = pick((a).F);                         \
    switch (c.L * 10 + c.NV) {                         \
      case 41: FN<4, 1>(a, s); break;                  \
      case 81: FN<8, 1>(a, s); break;                  \
      case 161: FN<16, 1>(a, s); break;                \
      case 321: FN<32, 1>(a, s); break;                \
      case 641: FN<64, 1>(a, s); break;                \
      case 642: FN<64, 2>(a, s); break;                \
      default: FN<64, 4>(a, s); break;                 \
    }                                                  \
  } while (0)

}  // namespace

bool gat_supported(int64_t H, int64_t D) {
  if (H < 1 || D < 4 || D % 4 != 0) return false;
  const int64_t d4 = D / 4;
  if ((d4 & (d4 - 1)) != 0) return false;       // head lanes reduce by xor-shuffle
  const int64_t F = H * D;
  if (F > 1024) return false;
  return d4 <= pick(F).L;
}

int64_t gat_chunk_edges(int64_t nnz) { return fast_chunk_edges(nnz, 64); }

void launch_gat_forward(const GatArgs& a, hipStream_t s) { DGLMI_GAT_DISPATCH(fwd_cfg, a, s); }
void launch_gat_merge(const float* out_part, const float* m_part, const float* l_part, int nb,
                      int64_t num_rows, int H, int D, float* out, float* m, float* l, hipStream_t s,
                      const float* lf_part, const float* ls_part, float* lf, float* ls) {
  const int64_t total = num_rows * (static_cast<int64_t>(H) * D / 4);
  if (total <= 0) return;
  const int64_t want = (total + kBlock - 1) / kBlock;
  const unsigned blocks = static_cast<unsigned>(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(k_gat_merge, dim3(blocks), dim3(kBlock), 0, s, out_part, m_part, l_part, nb,
                     num_rows, H, D, out, m, l, lf_part, ls_part, lf, ls);
}
// l[i] = m[i] + log(l[i]): the softmax state of a row as one log-sum-exp, so the
// backward's attention exp(s - m) / l becomes exp(s - lse) / 1 (the reference-order
// entry point when its (E, H) exp buffer is too small to hold the running max).
__global__ void k_gat_fold_lse(const float* __restrict__ m, float* __restrict__ l, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    l[i] = m[i] + logf(l[i]);
}
void launch_gat_fold_lse(const float* m, float* l, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  const unsigned blocks = static_cast<unsigned>(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(k_gat_fold_lse, dim3(blocks), dim3(kBlock), 0, s, m, l, n);
}

// GATConv's attention logits (gatconv.py:137-138 of the reference: el = (ft_src *
// attn_l).sum(-1), er = (ft_dst * attn_r).sum(-1)) in one pass over the projected
// features instead of torch's multiply + reduce per side (two reads of the (N, H, D)
// table and an (N, H, D) temporary each).  One thread per float4 slot of a row; the D4 =
// D / 4 slots of a head sit on adjacent, D4-aligned lanes (F4 = H D4 slots per row, D4 a
// power of two dividing 64), so a head's dot product is one xor butterfly over its
// lanes.  A D4-lane group is active or inactive as a whole (the bound is a whole row), so
// the butterfly only reads active lanes.  xs == xd (one feature table): read once.
// Summation order: torch's (x * a).sum(-1) on this device adds the rounded products as a
// pairwise tree of adjacent pairs ((p0 + p1) + (p2 + p3)) + ... (bit-for-bit on every
// element for D = 4 .. 64, the head sizes taken here: scripts/sum_order_probe.py, profiles/r06_sum_order_probe.jsonl);
// a lane's quad is the tree's first two levels and the butterfly over adjacent lanes the
// rest, so el / er are torch's bits -- the LeakyReLU of el + er takes the same branch as
// in the reference's composition.
__global__ void k_gat_logits(const float* __restrict__ xs, const float* __restrict__ xd, int64_t ns,
                             int64_t nd, int H, int D4, const float* __restrict__ al,
                             const float* __restrict__ ar, float* __restrict__ el,
                             float* __restrict__ er) {
  const int64_t F4 = static_cast<int64_t>(H) * D4;
  const int64_t rows = ns > nd ? ns : nd;
  const int64_t total = rows * F4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / F4;
    const int f4 = static_cast<int>(i - r * F4);
    const float4 a = ld4g(al + 4 * f4), b = ld4g(ar + 4 * f4);
    float sl = 0.0f, sr = 0.0f;
    if (r < ns) {
      const float4 x = ld4g(xs + r * F4 * 4 + 4 * f4);
      sl = (x.x * a.x + x.y * a.y) + (x.z * a.z + x.w * a.w);
      if (xd == xs) sr = (x.x * b.x + x.y * b.y) + (x.z * b.z + x.w * b.w);
    }
    if (xd != xs && r < nd) {
      const float4 y = ld4g(xd + r * F4 * 4 + 4 * f4);
      sr = (y.x * b.x + y.y * b.y) + (y.z * b.z + y.w * b.w);
    }
    for (int o = 1; o < D4; o <<= 1) {
      sl += __shfl_xor(sl, o);
      sr += __shfl_xor(sr, o);
    }
    if (f4 % D4 == 0) {
      const int64_t hi = r * H + f4 / D4;
      if (r < ns) el[hi] = sl;
      if (r < nd) er[hi] = sr;
    }
  }
}

// Its backward: grad_xs = g_el attn_l, grad_xd = g_er attn_r (one table: their sum, one
// write), and the parameter gradients sum_rows g_el xs / g_er xd as per-thread partials
// part[t] = {attn_l slot (4), attn_r slot (4)} -- the grid stride is a multiple of F4, so
// a thread's slot is fixed over its rows; the host sums the partials of each slot in
// thread order (a fixed grid for a given shape: deterministic).
__global__ void k_gat_logits_bwd(const float* __restrict__ xs, const float* __restrict__ xd, int64_t ns,
                                 int64_t nd, int H, int D4, const float* __restrict__ al,
                                 const float* __restrict__ ar, const float* __restrict__ gel,
                                 const float* __restrict__ ger, float* __restrict__ gs,
                                 float* __restrict__ gd, float* __restrict__ part) {
  const int64_t F4 = static_cast<int64_t>(H) * D4;
  const int64_t rows = ns > nd ? ns : nd;
  const int64_t total = rows * F4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int f4 = static_cast<int>(t % F4);
  const float4 a = ld4g(al + 4 * f4), b = ld4g(ar + 4 * f4);
  const int h = f4 / D4;
  float4 pl = make_float4(0.f, 0.f, 0.f, 0.f), pr = pl;
  const bool one = xd == xs;
  for (int64_t i = t; i < total; i += stride) {
    const int64_t r = i / F4;
    const int64_t o = r * F4 * 4 + 4 * f4;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < ns) {
      const float e = gel[r * H + h];
      const float4 x = ld4g(xs + o);
      g = make_float4(e * a.x, e * a.y, e * a.z, e * a.w);
      pl = make_float4(pl.x + e * x.x, pl.y + e * x.y, pl.z + e * x.z, pl.w + e * x.w);
      if (one) {
        const float q = ger[r * H + h];
        g = make_float4(g.x + q * b.x, g.y + q * b.y, g.z + q * b.z, g.w + q * b.w);
        pr = make_float4(pr.x + q * x.x, pr.y + q * x.y, pr.z + q * x.z, pr.w + q * x.w);
      }
      st4g(gs + o, g);
    }
    if (!one && r < nd) {
      const float q = ger[r * H + h];
      const float4 y = ld4g(xd + o);
      st4g(gd + o, make_float4(q * b.x, q * b.y, q * b.z, q * b.w));
      pr = make_float4(pr.x + q * y.x, pr.y + q * y.y, pr.z + q * y.z, pr.w + q * y.w);
    }
  }
  st4g(part + 8 * t, pl);
  st4g(part + 8 * t + 4, pr);
}

bool gat_logits_supported(int64_t H, int64_t D) {
  if (H < 1 || D < 4 || D % 4 != 0) return false;
  const int64_t D4 = D / 4, F4 = H * D4;
  // D <= 64: where torch's summation order was checked bit for bit (the header above)
  return (D4 & (D4 - 1)) == 0 && D4 <= 16 && F4 <= kBlock && kBlock % F4 == 0;
}
// threads of the logits kernels: whole blocks, at most 1024 of them (fixed for a shape)
int64_t gat_logits_threads(int64_t ns, int64_t nd, int64_t H, int64_t D) {
  const int64_t total = (ns > nd ? ns : nd) * H * (D / 4);
  int64_t blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  return blocks * kBlock;
}
void launch_gat_logits(const float* xs, const float* xd, int64_t ns, int64_t nd, int H, int D,
                       const float* al, const float* ar, float* el, float* er, hipStream_t s) {
  if (ns <= 0 && nd <= 0) return;
  const unsigned blocks = static_cast<unsigned>(gat_logits_threads(ns, nd, H, D) / kBlock);
  hipLaunchKernelGGL(k_gat_logits, dim3(blocks), dim3(kBlock), 0, s, xs, xd, ns, nd, H, D / 4, al, ar,
                     el, er);
}
void launch_gat_logits_bwd(const float* xs, const float* xd, int64_t ns, int64_t nd, int H, int D,
                           const float* al, const float* ar, const float* gel, const float* ger,
                           float* gs, float* gd, float* part, hipStream_t s) {
  const unsigned blocks = static_cast<unsigned>(gat_logits_threads(ns, nd, H, D) / kBlock);
  hipLaunchKernelGGL(k_gat_logits_bwd, dim3(blocks), dim3(kBlock), 0, s, xs, xd, ns, nd, H, D / 4, al,
                     ar, gel, ger, gs, gd, part);
}
// One keep word per edge from a dropout output (E, H) in edge-id order: the lanes of a
// wave read 64 consecutive rows, every byte of the span used over the H loads.
template <typename T>
__global__ void k_gat_keep_bits(const float* __restrict__ table, int64_t n, int H, T* __restrict__ bits) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t w = 0;
    for (int h = 0; h < H; ++h) w |= (table[e * H + h] != 0.0f ? 1u : 0u) << h;
    bits[e] = static_cast<T>(w);
  }
}
__global__ void k_dropout_draw_mask(uint64_t seed, uint64_t ctr, int64_t threads, int vec, int shift, float keep,
                                    int64_t n, uint8_t* __restrict__ mask) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const DrawSlot s = dropout_draw_slot(i, vec, threads, shift);
    mask[i] = dropout_draw_kept(dropout_draw(seed, ctr, s), s.comp, keep) ? 1 : 0;
  }
}
void launch_dropout_draw_mask(uint64_t seed, uint64_t ctr, int64_t threads, int vec, int shift, float keep,
                              int64_t n, uint8_t* mask, hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_dropout_draw_mask, dim3(static_cast<unsigned>(want < 65536 ? want : 65536)), dim3(kBlock),
                     0, s, seed, ctr, threads, vec, shift, keep, n, mask);
}
template <bool APPLY>
__global__ void k_dropout_draw_scale(GatArgs a, const int32_t* __restrict__ eids, int64_t n, float* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < n; p += stride) {
    const uint32_t kb = gat_draw_keep(a, eids != nullptr ? eids[p] : static_cast<int32_t>(p));
    for (int h = 0; h < a.H; ++h) {
      const float f = (kb >> h) & 1u ? a.drop_scale : 0.0f;
      if (APPLY) out[p * a.H + h] *= f;  // x * (1 * keep * scale): the composition's order
      else out[p * a.H + h] = f;
    }
  }
}
void launch_dropout_draw_scale(const GatArgs& a, const int32_t* eids, int64_t n, float* out, bool apply,
                               hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  const dim3 grid(static_cast<unsigned>(want < 65536 ? want : 65536)), blk(kBlock);
  if (apply) hipLaunchKernelGGL(k_dropout_draw_scale<true>, grid, blk, 0, s, a, eids, n, out);
  else hipLaunchKernelGGL(k_dropout_draw_scale<false>, grid, blk, 0, s, a, eids, n, out);
}
// The same from the dropout's own mask (E, H) bytes, 1 = kept (torch.native_dropout's
// second output): a quarter of the table's bytes.  H = 8 (the reference GAT's heads) reads
// a row as one 8-byte load.
template <typename T>
__global__ void k_gat_keep_bits_mask(const uint8_t* __restrict__ mask, int64_t n, int H, T* __restrict__ bits) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t w = 0;
    if (H == 8) {
      const uint64_t v = reinterpret_cast<const uint64_t*>(mask)[e];
#pragma unroll
      for (int h = 0; h < 8; ++h) w |= (((v >> (8 * h)) & 0xffu) != 0 ? 1u : 0u) << h;
    } else {
      for (int h = 0; h < H; ++h) w |= (mask[e * H + h] != 0 ? 1u : 0u) << h;
    }
    bits[e] = static_cast<T>(w);
  }
}
void launch_gat_keep_bits_mask(const uint8_t* mask, int64_t n, int H, void* bits, int width, hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  const dim3 grid(static_cast<unsigned>(want < 65536 ? want : 65536)), blk(kBlock);
  if (width == 8)
    hipLaunchKernelGGL(k_gat_keep_bits_mask<uint8_t>, grid, blk, 0, s, mask, n, H, static_cast<uint8_t*>(bits));
  else if (width == 16)
    hipLaunchKernelGGL(k_gat_keep_bits_mask<uint16_t>, grid, blk, 0, s, mask, n, H, static_cast<uint16_t*>(bits));
  else
    hipLaunchKernelGGL(k_gat_keep_bits_mask<uint32_t>, grid, blk, 0, s, mask, n, H, static_cast<uint32_t*>(bits));
}
void launch_gat_keep_bits(const float* table, int64_t n, int H, void* bits, int width, hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  const dim3 grid(static_cast<unsigned>(want < 65536 ? want : 65536)), blk(kBlock);
  if (width == 8)
    hipLaunchKernelGGL(k_gat_keep_bits<uint8_t>, grid, blk, 0, s, table, n, H, static_cast<uint8_t*>(bits));
  else if (width == 16)
    hipLaunchKernelGGL(k_gat_keep_bits<uint16_t>, grid, blk, 0, s, table, n, H, static_cast<uint16_t*>(bits));
  else
    hipLaunchKernelGGL(k_gat_keep_bits<uint32_t>, grid, blk, 0, s, table, n, H, static_cast<uint32_t*>(bits));
}
template <typename T>
__global__ void k_gat_keep_gather(const T* __restrict__ keep, const int32_t* __restrict__ index, int64_t n,
                                  T* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = keep[index[i]];
}
void launch_gat_keep_gather(const void* keep, int width, const int32_t* index, int64_t n, void* out,
                            hipStream_t s) {
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  const dim3 grid(static_cast<unsigned>(want < 65536 ? want : 65536)), blk(kBlock);
  if (width == 8)
    hipLaunchKernelGGL(k_gat_keep_gather<uint8_t>, grid, blk, 0, s, static_cast<const uint8_t*>(keep), index, n,
                       static_cast<uint8_t*>(out));
  else if (width == 16)
    hipLaunchKernelGGL(k_gat_keep_gather<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(keep), index,
                       n, static_cast<uint16_t*>(out));
  else
    hipLaunchKernelGGL(k_gat_keep_gather<uint32_t>, grid, blk, 0, s, static_cast<const uint32_t*>(keep), index,
                       n, static_cast<uint32_t*>(out));
}
void launch_gat_backward_dst(const GatArgs& a, hipStream_t s) { DGLMI_GAT_DISPATCH(bwd_dst_cfg, a, s); }
void launch_gat_backward_src(const GatArgs& a, hipStream_t s) { DGLMI_GAT_DISPATCH(bwd_src_cfg, a, s); }
void launch_gat_stats(const GatArgs& a, hipStream_t s) {
  const int64_t n = a.num_rows * (a.F / 4);
  if (n <= 0) return;
  const int64_t want = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_gat_stats, dim3(static_cast<unsigned>(want < 65536 ? want : 65536)),
                     dim3(kBlock), 0, s, a);
}

}  // namespace dglmi
