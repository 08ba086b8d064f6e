// Bracketing projections Y = X W (+ b) for gfx950 on v_mfma_f32_16x16x4_f32, for the
// tall-skinny shapes GraphConv / GATConv / RelGraphConv project node features with
// (M node rows >> K, N; fp32 like the reference's torch.matmul, graphconv.py:146-170,
// gatconv.py:127-132, relgraphconv.py).
//
// Two kernels, one operand layout.  Inside each 16-k block lane group g takes k = 4g + s
// at MFMA step s, so a lane's four X values are one float4; W goes in as the MFMA's A
// operand, so the accumulator is Y's transpose and each lane ends with four consecutive
// columns of one row (one float4 store per 16-column block).  W stays in the waves'
// registers for the whole (persistent) launch; X streams once.
//
// * k_project (K in {16, 32, 64, 128}, N in {64, 128}): a wave owns 16 rows x 64 columns
//   and streams its X rows itself as float4, two tiles ahead.  C2 shape (169 343 x 128 ->
//   128): 66.7 us against 111.2 us for torch.matmul (hipBLASLt), scripts/gemm_ts_probe.hip.
// * k_project_tile (any K <= 640, any N): the four waves of a workgroup share each
//   16-row X tile, staged through LDS from its contiguous 16 K-float span (coalesced
//   float4 loads of any row width, zero-padded to the padded K), double-buffered; the
//   waves split the tile's work NS column slices x KS k-slices.  NS = 4 gives wide outputs
//   (R-GCN's 64 -> 4 x 64 relation-major projection) ONE X read for all their columns
//   where k_project re-read X per 64-column slice; KS = 4 splits a long K (GATConv's
//   602 -> 64 on Reddit) over the waves' registers, the partial tiles summed through LDS.
#include "internal.h"

#include <algorithm>
#include <cstdlib>

namespace dglmi {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kNW = 64;       // columns per wave
constexpr int kWaves = 4;     // waves per workgroup (one column slice)

template <int K>
__global__ void __launch_bounds__(64 * kWaves) k_project(const float* __restrict__ X, const float* __restrict__ W,
                                                         int64_t swk, int64_t swn, const float* __restrict__ bias,
                                                         float* __restrict__ Y, int64_t M, int64_t N) {
  constexpr int KB = K / 16;    // 16-k blocks
  constexpr int CB = kNW / 16;  // 16-column blocks per wave
  __shared__ float sW[K][kNW + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t slices = N / kNW;
  const int64_t rtiles = (M + 15) / 16;
  const int64_t n0 = (blockIdx.x % slices) * kNW;
  // W[:, n0 : n0 + 64] into LDS, the unit-stride dimension fastest
  for (int i = threadIdx.x; i < K * kNW; i += 64 * kWaves) {
    const int k = swk == 1 ? i % K : i / kNW;
    const int n = swk == 1 ? i / K : i % kNW;
    sW[k][n] = W[k * swk + (n0 + n) * swn];
  }
  __syncthreads();
  float w[KB][4][CB];
#pragma unroll
  for (int q = 0; q < KB; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < CB; ++c) w[q][s][c] = sW[16 * q + 4 * g + s][16 * c + r];
  float4 bv[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c)
    bv[c] = bias ? *reinterpret_cast<const float4*>(bias + n0 + 16 * c + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  // row tiles of this slice: wave w of workgroup j takes (j / slices) * 4 + w, then + step
  const int64_t groups = gridDim.x / slices;
  const int64_t step = groups * kWaves;
  int64_t t = (blockIdx.x / slices) * kWaves + wv;
  if (t >= rtiles) return;
  auto load_x = [&](int64_t tt, float4 (&a)[KB]) {
    const int64_t row = tt * 16 + r;
#pragma unroll
    for (int q = 0; q < KB; ++q)
      a[q] = row < M ? *reinterpret_cast<const float4*>(X + row * K + 16 * q + 4 * g)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float4 a[KB], a1[KB], a2[KB];
  load_x(t, a);
  if (t + step < rtiles) load_x(t + step, a1);
  for (; t < rtiles; t += step) {
    if (t + 2 * step < rtiles) load_x(t + 2 * step, a2);
    f4v acc[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[c] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const float av[4] = {a[q].x, a[q].y, a[q].z, a[q].w};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[q][s][c], av[s], acc[c], 0, 0, 0);
    }
    const int64_t row = t * 16 + r;
    if (row < M) {
#pragma unroll
      for (int c = 0; c < CB; ++c)
        *reinterpret_cast<float4*>(Y + row * N + n0 + 16 * c + 4 * g) =
            make_float4(acc[c][0] + bv[c].x, acc[c][1] + bv[c].y, acc[c][2] + bv[c].z, acc[c][3] + bv[c].w);
    }
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      a[q] = a1[q];
      a1[q] = a2[q];
    }
  }
}

// ---------------------------------------------------------------------------
// k_project_tile<KB, CB, NS, RAW>: wave (ni, ki) of the workgroup (ni < NS, ki < KS = 4 /
// NS) multiplies k in [16 KB ki, 16 KB (ki + 1)) into columns [16 CB ni, 16 CB (ni + 1))
// of the workgroup's column slice (NS 16 CB columns; columns past N come from zero W
// and are not stored); the padded K is KP = 16 KB KS (W rows past K are zero).  X tile
// image in LDS, by K's alignment:
//   RAW = 0 (K % 4 == 0): rows of KP + 4 floats (16 B apart in the banks), zero columns
//     K..KP, fragments by ds_read_b128;
//   RAW = 1 / 2 (K odd / K % 4 == 2, e.g. GATConv's 602): the contiguous span itself,
//     rows K floats apart -- staged by plain ds_write_b128, no per-element row split --
//     read as 4 ds_read_b32 / 2 ds_read_b64 per fragment, the k-block that straddles K
//     masked in registers (the next row's floats are not zero).
// ---------------------------------------------------------------------------
template <int KB, int CB, int NS>
struct TileShape {
  static constexpr int KS = kWaves / NS;
  static constexpr int KW = 16 * KB;           // k per wave
  static constexpr int KP = KS * KW;           // padded K
  static constexpr int LROW = KP + 4;          // padded row stride (floats, RAW = 0)
  static constexpr int NWC = 16 * CB;          // columns per wave
  static constexpr int NSL = NS * NWC;         // columns per workgroup slice
  static constexpr int NJ = (4 * KP + 255) / 256;  // float4 staging loads per thread per tile (16 KP / 4 / 256)
  static constexpr int NRED = KS > 1 ? (KS - 1) * NS : 0;
  static constexpr int NACC = CB <= 2 ? 2 : 1;  // accumulator sets: short chains alternate two
  // ONE __shared__ array (a second LDS object made hipcc wait vmcnt(0) -- for the next
  // tile's loads -- before the first ds_read of every tile): [X buffer 0][X buffer 1]
  // [partial accumulators of the waves ki > 0: NRED x CB x 64 float4][bias of the slice]
  static constexpr int XBUF = 16 * LROW + 16;  // + slack: a RAW read past the last row's end (masked)
  static constexpr int RED_OFF = 2 * XBUF;
  static constexpr int BIAS_OFF = RED_OFF + NRED * CB * 64 * 4;
  static constexpr int FLOATS = BIAS_OFF + NSL;
};

template <int KB, int CB, int NS, int RAW, int OCC>
__global__ void __launch_bounds__(64 * kWaves, OCC)
    k_project_tile(const float* __restrict__ X, int64_t M, int K, const float* __restrict__ W, int64_t swk,
                   int64_t swn, int64_t N, const float* __restrict__ bias, float* __restrict__ Y, int64_t slices) {
  using S = TileShape<KB, CB, NS>;
  __shared__ __attribute__((aligned(16))) float smem[S::FLOATS];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int ni = wv % NS, ki = wv / NS;
  const int r = lane & 15, g = lane >> 4;
  const int ls = RAW ? K : S::LROW;           // image row stride (floats)
  const int64_t slice = blockIdx.x % slices;
  const int64_t n_slice = slice * S::NSL;
  const int64_t nw0 = n_slice + ni * S::NWC;  // this wave's first column
  const int k0 = ki * S::KW;                  // this wave's first k
  const int64_t rtiles = (M + 15) / 16;
  const int64_t full = M / 16;                // tiles of 16 rows
  const int64_t groups = gridDim.x / slices;
  int64_t t = blockIdx.x / slices;
  // padded image: zero columns [K, KP) of both buffers once (tile loads write only k < K);
  // the slice's bias into LDS (0 past N or without bias)
  if (!RAW) {
    const int pad = S::KP - K;
    for (int i = tid; i < 32 * pad; i += 64 * kWaves)
      smem[(i / (16 * pad)) * S::XBUF + ((i / pad) % 16) * S::LROW + K + i % pad] = 0.0f;
  }
  for (int i = tid; i < S::NSL; i += 64 * kWaves)
    smem[S::BIAS_OFF + i] = (bias != nullptr && n_slice + i < N) ? bias[n_slice + i] : 0.0f;
  // this wave's W fragment, zero outside K x N (read once per workgroup; W is L2-resident)
  float w[KB][4][CB];
#pragma unroll
  for (int q = 0; q < KB; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int k = k0 + 16 * q + 4 * g + s;
        const int64_t n = nw0 + 16 * c + r;
        w[q][s][c] = (k < K && n < N) ? W[k * swk + n * swn] : 0.0f;
      }
  if (t >= rtiles) return;  // uniform over the workgroup (never taken: groups <= rtiles)
  // a tile's X rows are one contiguous span of 16 K floats, 16-byte aligned (X aligned);
  // thread tid stages float4s tid, tid + 256, ... of it
  const float invK = 1.0f / static_cast<float>(K);
  float4 st[S::NJ];
  // a whole tile: NJ unconditional float4 loads, all in flight at once behind the MFMAs
  // (a per-load bounds branch makes hipcc wait for every load); slots past the span
  // re-read its last float4 and are not stored
  auto load_full = [&](int64_t tt) {
    const float* base = X + tt * 16 * static_cast<int64_t>(K);
#pragma unroll
    for (int j = 0; j < S::NJ; ++j)
      st[j] = *reinterpret_cast<const float4*>(base + std::min(4 * (tid + 256 * j), 16 * K - 4));
  };
  // the last, partial tile (once per launch, off the pipelined path)
  auto load_part = [&](int64_t tt) {
    const float* base = X + tt * 16 * static_cast<int64_t>(K);
    const int avail = static_cast<int>(M - tt * 16) * K;
#pragma unroll
    for (int j = 0; j < S::NJ; ++j) {
      const int e = 4 * (tid + 256 * j);
      st[j].x = e < avail ? base[e] : 0.0f;
      st[j].y = e + 1 < avail ? base[e + 1] : 0.0f;
      st[j].z = e + 2 < avail ? base[e + 2] : 0.0f;
      st[j].w = e + 3 < avail ? base[e + 3] : 0.0f;
    }
  };
  auto store_tile = [&](int b) {
    float* sx = smem + b * S::XBUF;
#pragma unroll
    for (int j = 0; j < S::NJ; ++j) {
      const int e = 4 * (tid + 256 * j);
      if (e >= 16 * K) break;
      if (RAW) {  // the span itself
        *reinterpret_cast<float4*>(sx + e) = st[j];
        continue;
      }
      // K % 4 == 0: a float4 never straddles rows; its row e / K through the reciprocal
      // (exact: e + 0.5 is at least 0.5 / K away from a multiple of K)
      const int row = static_cast<int>((static_cast<float>(e) + 0.5f) * invK);
      *reinterpret_cast<float4*>(sx + row * S::LROW + (e - row * K)) = st[j];
    }
  };
  // lane (r, g)'s four X values of k-block q: k = k0 + 16 q + 4 g + s
  auto frag = [&](const float* sx, int q) -> f4v {
    const float* p = sx + r * ls + k0 + 16 * q + 4 * g;
    f4v x;
    if (RAW == 0) {
      x = *reinterpret_cast<const f4v*>(p);
    } else if (RAW == 2) {
      const float2 lo = *reinterpret_cast<const float2*>(p), hi = *reinterpret_cast<const float2*>(p + 2);
      x = f4v{lo.x, lo.y, hi.x, hi.y};
    } else {
      x = f4v{p[0], p[1], p[2], p[3]};
    }
    if (RAW && k0 + 16 * q + 16 > K) {  // the block that straddles K: the next row's floats
      const int kk = k0 + 16 * q + 4 * g;
#pragma unroll
      for (int s = 0; s < 4; ++s) x[s] = kk + s < K ? x[s] : 0.0f;
    }
    return x;
  };
  if (t < full) load_full(t); else load_part(t);
  store_tile(0);
  __syncthreads();
  int cur = 0;
  for (; t < rtiles; t += groups) {
    const int64_t tn = t + groups;
    // unconditional (past the last whole tile it re-reads that tile, unused): a load
    // under a branch made hipcc drain vmcnt(0) -- these loads included -- before the
    // MFMAs, for the previous tile's stores; straight-line, it counts them instead
    load_full(tn < full ? tn : full - 1);  // in flight during this tile's MFMAs
    const float* sx = smem + cur * S::XBUF;
    f4v acc[S::NACC][CB];
#pragma unroll
    for (int h = 0; h < S::NACC; ++h)
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[h][c] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const f4v xa = frag(sx, q);
      f4v* ac = acc[S::NACC == 2 ? (q & 1) : 0];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < CB; ++c) ac[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[q][s][c], xa[s], ac[c], 0, 0, 0);
    }
    if constexpr (S::NACC == 2) {
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[0][c] += acc[1][c];
    }
    if constexpr (S::KS > 1) {
      f4v* red = reinterpret_cast<f4v*>(smem + S::RED_OFF);
      if (ki > 0) {
#pragma unroll
        for (int c = 0; c < CB; ++c) red[(((ki - 1) * NS + ni) * CB + c) * 64 + lane] = acc[0][c];
      }
      __syncthreads();
      if (ki == 0) {
#pragma unroll
        for (int j = 1; j < S::KS; ++j)
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[0][c] += red[(((j - 1) * NS + ni) * CB + c) * 64 + lane];
      }
    }
    const int64_t row = t * 16 + r;
    if (ki == 0 && row < M) {
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int nl = ni * S::NWC + 16 * c + 4 * g;  // column within the slice
        const int64_t n = n_slice + nl;
        const f4v bv = *reinterpret_cast<const f4v*>(smem + S::BIAS_OFF + nl);
        const f4v o = acc[0][c] + bv;
        float* y = Y + row * N + n;
        if ((N & 3) == 0) {
          if (n < N) *reinterpret_cast<float4*>(y) = make_float4(o[0], o[1], o[2], o[3]);
        } else if ((N & 1) == 0) {
          if (n < N) *reinterpret_cast<float2*>(y) = make_float2(o[0], o[1]);
          if (n + 2 < N) *reinterpret_cast<float2*>(y + 2) = make_float2(o[2], o[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n + j < N) y[j] = o[j];
        }
      }
    }
    if (tn < rtiles) {
      if (tn >= full) load_part(tn);  // the partial last tile: loaded here, once
      store_tile(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------
// k_project_glds<KB, CB, NS>: the RAW layout (K % 4 != 0) with the X tiles copied global
// -> LDS by the LDS-DMA loads (global_load_lds_dwordx4: no staging registers, no write
// pass), three buffers, two tiles in flight across the barriers.  A tile's span is 16 K
// floats; every wave copies GW 1-KiB chunks of it per tile (a fixed count, so the wait
// for the tile two loads back is one counted vmcnt(GW)); the source addresses are
// clamped to the matrix, so the chunks past the span and the last, partial tile need no
// branch (rows past M are computed and not stored) -- except the tile holding X's end
// when M K is not a multiple of 4, copied 4 bytes at a time (the vmcnt(GW) after it waits
// for more than it must: correct).  The barriers are raw s_barrier
// after explicit waits: __syncthreads() would drain the in-flight copies (vmcnt(0)).
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_void_ptr;

template <int KB, int CB, int NS>
struct GldsShape {
  using T = TileShape<KB, CB, NS>;
  static constexpr int GW = (T::KP + 63) / 64;          // 1-KiB chunks per wave per tile
  static constexpr int XBUF = kWaves * GW * 256 + 16;   // floats per buffer (+ slack past the last row)
  static constexpr int RED_OFF = 3 * XBUF;
  static constexpr int BIAS_OFF = RED_OFF + T::NRED * CB * 64 * 4;
  static constexpr int FLOATS = BIAS_OFF + T::NSL;
};

template <int KB, int CB, int NS, int RAW>
__global__ void __launch_bounds__(64 * kWaves, 1)
    k_project_glds(const float* __restrict__ X, int64_t M, int K, const float* __restrict__ W, int64_t swk,
                   int64_t swn, int64_t N, const float* __restrict__ bias, float* __restrict__ Y, int64_t slices) {
  using S = TileShape<KB, CB, NS>;
  using G = GldsShape<KB, CB, NS>;
  __shared__ __attribute__((aligned(16))) float smem[G::FLOATS];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int ni = wv % NS, ki = wv / NS;
  const int r = lane & 15, g = lane >> 4;
  const int64_t slice = blockIdx.x % slices;
  const int64_t n_slice = slice * S::NSL;
  const int64_t nw0 = n_slice + ni * S::NWC;
  const int k0 = ki * S::KW;
  const int64_t rtiles = (M + 15) / 16;
  const int64_t groups = gridDim.x / slices;
  const int64_t total = M * static_cast<int64_t>(K);
  const int64_t last = (total & ~int64_t(3)) - 4;  // the last whole, aligned float4 (M >= 16)
  int64_t t = blockIdx.x / slices;
  for (int i = tid; i < S::NSL; i += 64 * kWaves)
    smem[G::BIAS_OFF + i] = (bias != nullptr && n_slice + i < N) ? bias[n_slice + i] : 0.0f;
  float w[KB][4][CB];
#pragma unroll
  for (int q = 0; q < KB; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int k = k0 + 16 * q + 4 * g + s;
        const int64_t n = nw0 + 16 * c + r;
        w[q][s][c] = (k < K && n < N) ? W[k * swk + n * swn] : 0.0f;
      }
  // the W loads are consumed before the first copy is in flight (a use of an ordinary
  // load's result while a copy is outstanding makes hipcc drain every copy)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (t >= rtiles) return;
  // tile tt's GW chunks of this wave into buffer b (tile index clamped: past the end the
  // copy re-reads the last tile into a buffer that is never read)
  // (dst: the buffer; a __restrict__ parameter, so that the copy and the reads of the
  // other buffer carry disjoint alias scopes -- without them hipcc waits vmcnt(0) for
  // every copy in flight before each LDS read)
  auto copy_tile = [&](int64_t tt, float* __restrict__ dst) {
    tt = tt < rtiles ? tt : rtiles - 1;
    const int64_t base = tt * 16 * static_cast<int64_t>(K);
    if (tt == rtiles - 1 && (total & 3) != 0) {
      // the tile holding X's end when M K is not a multiple of 4: 4-byte copies clamped
      // to the last float (a 16-byte one would read past the matrix); once per launch
#pragma unroll
      for (int i = 0; i < 4 * G::GW; ++i) {
        const int piece = wv * 4 * G::GW + i;  // 64 floats
        const int64_t e = std::min<int64_t>(base + piece * 64 + lane, total - 1);
        __builtin_amdgcn_global_load_lds(X + e, (lds_void_ptr)(dst + piece * 64), 4, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < G::GW; ++i) {
      const int chunk = wv * G::GW + i;
      const int64_t e = std::min<int64_t>(base + chunk * 256 + lane * 4, last);
      __builtin_amdgcn_global_load_lds(X + e, (lds_void_ptr)(dst + chunk * 256), 16, 0, 0);
    }
  };
  auto frag = [&](const float* __restrict__ sx, int q) -> f4v {
    const float* p = sx + r * K + k0 + 16 * q + 4 * g;
    f4v x;
    if (RAW == 2) {
      const float2 lo = *reinterpret_cast<const float2*>(p), hi = *reinterpret_cast<const float2*>(p + 2);
      x = f4v{lo.x, lo.y, hi.x, hi.y};
    } else {
      x = f4v{p[0], p[1], p[2], p[3]};
    }
    if (k0 + 16 * q + 16 > K) {  // the block that straddles K: the next row's floats
      const int kk = k0 + 16 * q + 4 * g;
#pragma unroll
      for (int s = 0; s < 4; ++s) x[s] = kk + s < K ? x[s] : 0.0f;
    }
    return x;
  };
  copy_tile(t, smem);
  copy_tile(t + groups, smem + G::XBUF);
  // one tile: the copy of tile t + 2 groups into `next`, the MFMAs over `sx` (restrict:
  // disjoint alias scopes for the copy and the reads)
  auto step = [&](int64_t t, const float* __restrict__ sx, float* __restrict__ next) {
    copy_tile(t + 2 * groups, next);
    f4v acc[S::NACC][CB];
#pragma unroll
    for (int h = 0; h < S::NACC; ++h)
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[h][c] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const f4v xa = frag(sx, q);
      f4v* ac = acc[S::NACC == 2 ? (q & 1) : 0];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < CB; ++c) ac[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[q][s][c], xa[s], ac[c], 0, 0, 0);
    }
    if constexpr (S::NACC == 2) {
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[0][c] += acc[1][c];
    }
    if constexpr (S::KS > 1) {
      f4v* red = reinterpret_cast<f4v*>(smem + G::RED_OFF);
      if (ki > 0) {
#pragma unroll
        for (int c = 0; c < CB; ++c) red[(((ki - 1) * NS + ni) * CB + c) * 64 + lane] = acc[0][c];
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (ki == 0) {
#pragma unroll
        for (int j = 1; j < S::KS; ++j)
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[0][c] += red[(((j - 1) * NS + ni) * CB + c) * 64 + lane];
      }
    }
    const int64_t row = t * 16 + r;
    if (ki == 0 && row < M) {
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int nl = ni * S::NWC + 16 * c + 4 * g;
        const int64_t n = n_slice + nl;
        const f4v bv = *reinterpret_cast<const f4v*>(smem + G::BIAS_OFF + nl);
        const f4v o = acc[0][c] + bv;
        float* y = Y + row * N + n;
        if ((N & 3) == 0) {
          if (n < N) *reinterpret_cast<float4*>(y) = make_float4(o[0], o[1], o[2], o[3]);
        } else if ((N & 1) == 0) {
          if (n < N) *reinterpret_cast<float2*>(y) = make_float2(o[0], o[1]);
          if (n + 2 < N) *reinterpret_cast<float2*>(y + 2) = make_float2(o[2], o[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n + j < N) y[j] = o[j];
        }
      }
    }
  };
  int b = 0;
  for (; t < rtiles; t += groups) {
    // this wave's copies of tile t are done (the GW after them may be in flight), then
    // every wave's are; the buffer the next copy overwrites was read one tile ago
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(G::GW) : "memory");
    step(t, smem + b * G::XBUF, smem + (b == 0 ? 2 : b - 1) * G::XBUF);
    b = b == 2 ? 0 : b + 1;
  }
  // drain the copies still in flight (clamped re-reads) before the workgroup ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the k_project_tile instances, by padded K and slice width
struct TileCfg {
  int KB, CB, NS;
  int kp() const { return (kWaves / NS) * 16 * KB; }
  int nsl() const { return NS * 16 * CB; }
};
constexpr TileCfg kTileCfgs[] = {
    {1, 4, 4},   // K <= 16,  N <= 256
    {2, 4, 4},   // K <= 32,  N <= 256
    {4, 4, 4},   // K <= 64,  N <= 256  (R-GCN 64 -> 4 x 64 relation-major)
    {4, 10, 4},  // K <= 64,  N <= 640  (GATConv's dX: 64 -> 602)
    {4, 4, 2},   // K <= 128, N <= 128
    {8, 4, 2},   // K <= 256, N <= 128
    {16, 1, 4},  // K <= 256, N <= 64   (R-GCN dX: 256 -> 64), no k split
    {8, 4, 1},   // K <= 512, N <= 64
    {40, 1, 4},  // K <= 640, N <= 64   (GATConv 602 -> 8 x 8 on Reddit), no k split
    {4, 4, 1},   // K <= 256, N <= 64   (k split; A/B)
    {10, 4, 1},  // K <= 640, N <= 64   (k split: GATConv 602 -> 8 x 8, 0.24 vs 0.34 ms)
    {4, 5, 4},   // K <= 64,  N <= 320  (two column slices of GATConv's dX; A/B)
};
constexpr int kNumTileCfgs = sizeof(kTileCfgs) / sizeof(kTileCfgs[0]);

// the instance with the least padded MFMA work for (K, N) (X re-reads of extra column
// slices priced at 10 % each, a k split's LDS reduction at 5 %, and a wave that reads a
// whole tile of more than 256 k from LDS -- four times the LDS reads of the k split -- at
// 50 %: C3's 602 -> 64 runs 0.34 ms that way against 0.24 ms split, while C5's 256 -> 64
// runs 1.58 ms unsplit against 1.85 ms split; scripts/project_probe.py); -1: none (K > 640).
// DGLMI_PROJECT_CFG=i forces instance i where it fits (A/B).
int pick_tile(int64_t K, int64_t N) {
  if (const char* e = std::getenv("DGLMI_PROJECT_CFG")) {
    const int i = std::atoi(e);
    if (i >= 0 && i < kNumTileCfgs && K <= kTileCfgs[i].kp()) return i;
  }
  int best = -1;
  double best_cost = 0.0;
  for (int i = 0; i < kNumTileCfgs; ++i) {
    const TileCfg& c = kTileCfgs[i];
    if (K > c.kp()) continue;
    const int64_t slices = (N + c.nsl() - 1) / c.nsl();
    const double cost = static_cast<double>(c.kp()) * slices * c.nsl() * (1.0 + 0.1 * (slices - 1)) *
                        (c.NS < kWaves ? 1.05 : 1.0) * (c.NS == kWaves && 16 * c.KB > 256 ? 1.5 : 1.0);
    if (best < 0 || cost < best_cost) {
      best = i;
      best_cost = cost;
    }
  }
  return best;
}

template <int KB, int CB, int NS, int RAW>
void launch_tile_raw(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn, int64_t N,
                     const float* bias, float* Y, hipStream_t s) {
  using S = TileShape<KB, CB, NS>;
  // two workgroups per CU where the W fragment leaves room (<= 256 VGPRs per lane)
  constexpr int OCC = 4 * KB * CB <= 80 ? 2 : 1;
  const int64_t slices = (N + S::NSL - 1) / S::NSL;
  const int64_t rtiles = (M + 15) / 16;
  int64_t groups = std::max<int64_t>(1, 256 * OCC / slices);
  groups = std::min<int64_t>(groups, rtiles);
  hipLaunchKernelGGL((k_project_tile<KB, CB, NS, RAW, OCC>), dim3(static_cast<unsigned>(groups * slices)),
                     dim3(64 * kWaves), 0, s, X, M, static_cast<int>(K), W, swk, swn, N, bias, Y, slices);
}

template <int KB, int CB, int NS, int RAW>
void launch_glds(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn, int64_t N,
                 const float* bias, float* Y, hipStream_t s) {
  using S = TileShape<KB, CB, NS>;
  const int64_t slices = (N + S::NSL - 1) / S::NSL;
  const int64_t rtiles = (M + 15) / 16;
  int64_t groups = std::max<int64_t>(1, 256 / slices);
  groups = std::min<int64_t>(groups, rtiles);
  hipLaunchKernelGGL((k_project_glds<KB, CB, NS, RAW>), dim3(static_cast<unsigned>(groups * slices)),
                     dim3(64 * kWaves), 0, s, X, M, static_cast<int>(K), W, swk, swn, N, bias, Y, slices);
}

// DGLMI_PROJECT_GLDS=0 keeps the register-staged copy for the RAW layouts (A/B)
bool use_glds() {
  const char* e = std::getenv("DGLMI_PROJECT_GLDS");
  return e == nullptr || e[0] != '0';
}

template <int KB, int CB, int NS>
void launch_tile(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn, int64_t N,
                 const float* bias, float* Y, hipStream_t s) {
  // M >= 16 (the C entry checks): the in-loop prefetch re-reads the last whole tile
  if (K % 4 == 0) launch_tile_raw<KB, CB, NS, 0>(X, M, K, W, swk, swn, N, bias, Y, s);
  else if (use_glds() && K % 2 == 0) launch_glds<KB, CB, NS, 2>(X, M, K, W, swk, swn, N, bias, Y, s);
  else if (use_glds()) launch_glds<KB, CB, NS, 1>(X, M, K, W, swk, swn, N, bias, Y, s);
  else if (K % 2 == 0) launch_tile_raw<KB, CB, NS, 2>(X, M, K, W, swk, swn, N, bias, Y, s);
  else launch_tile_raw<KB, CB, NS, 1>(X, M, K, W, swk, swn, N, bias, Y, s);
}

// DGLMI_PROJECT_TILE=1 sends the shapes k_project covers to k_project_tile too (A/B)
bool force_tile() {
  const char* e = std::getenv("DGLMI_PROJECT_TILE");
  return e != nullptr && e[0] == '1';
}

}  // namespace

bool project_supported(int64_t K, int64_t N) { return K >= 1 && N >= 1 && N <= (1 << 20) && pick_tile(K, N) >= 0; }

void launch_project(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn,
                    int64_t N, const float* bias, float* Y, hipStream_t s) {
  if (M == 0) return;
  const bool direct = (K == 16 || K == 32 || K == 64 || K == 128) && (N == 64 || N == 128) && !force_tile();
  if (direct) {
    const int64_t slices = N / kNW;
    const int64_t rtiles = (M + 15) / 16;
    // one wave per SIMD over the chip (256 CUs x 4), split between the column slices
    int64_t groups = std::max<int64_t>(1, 256 / slices);
    groups = std::min<int64_t>(groups, (rtiles + kWaves - 1) / kWaves);
    const dim3 grid(static_cast<unsigned>(groups * slices)), blk(64 * kWaves);
    switch (K) {
      case 16: hipLaunchKernelGGL(k_project<16>, grid, blk, 0, s, X, W, swk, swn, bias, Y, M, N); break;
      case 32: hipLaunchKernelGGL(k_project<32>, grid, blk, 0, s, X, W, swk, swn, bias, Y, M, N); break;
      case 64: hipLaunchKernelGGL(k_project<64>, grid, blk, 0, s, X, W, swk, swn, bias, Y, M, N); break;
      default: hipLaunchKernelGGL(k_project<128>, grid, blk, 0, s, X, W, swk, swn, bias, Y, M, N); break;
    }
    return;
  }
  switch (pick_tile(K, N)) {
    case 0: launch_tile<1, 4, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 1: launch_tile<2, 4, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 2: launch_tile<4, 4, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 3: launch_tile<4, 10, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 4: launch_tile<4, 4, 2>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 5: launch_tile<8, 4, 2>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 6: launch_tile<16, 1, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 7: launch_tile<8, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 8: launch_tile<40, 1, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 9: launch_tile<4, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 10: launch_tile<10, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 11: launch_tile<4, 5, 4>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    default: break;  // unsupported: the C entry checks project_supported first
  }
}

}  // namespace dglmi
