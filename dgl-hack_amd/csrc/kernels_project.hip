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
// k_project_tile<KB, CB, NS>: wave (ni, ki) of the workgroup (ni < NS, ki < KS = 4 / NS)
// multiplies k in [16 KB ki, 16 KB (ki + 1)) into columns n0 + [16 CB ni, 16 CB (ni + 1))
// of the workgroup's column slice; the padded K is KP = 16 KB KS (zero rows of W and
// zero LDS columns past K), the slice is NS 16 CB columns wide (columns past N are
// computed from zero W and not stored).
// ---------------------------------------------------------------------------
template <int KB, int CB, int NS>
struct TileShape {
  static constexpr int KS = kWaves / NS;
  static constexpr int KW = 16 * KB;           // k per wave
  static constexpr int KP = KS * KW;           // padded K
  static constexpr int LROW = KP + 4;          // LDS row stride (floats): rows land 16 B apart in the banks
  static constexpr int NWC = 16 * CB;          // columns per wave
  static constexpr int NSL = NS * NWC;         // columns per workgroup slice
  static constexpr int NJ = (4 * KP + 255) / 256;  // float4 staging loads per thread per tile (16 KP / 4 / 256)
  static constexpr int NRED = KS > 1 ? (KS - 1) * NS : 1;
};

template <int KB, int CB, int NS, int OCC>
__global__ void __launch_bounds__(64 * kWaves, OCC)
    k_project_tile(const float* __restrict__ X, int64_t M, int K, const float* __restrict__ W, int64_t swk,
                   int64_t swn, int64_t N, const float* __restrict__ bias, float* __restrict__ Y, int64_t slices) {
  using S = TileShape<KB, CB, NS>;
  __shared__ __attribute__((aligned(16))) float sX[2][16][S::LROW];
  __shared__ f4v sRed[S::NRED][CB][64];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int ni = wv % NS, ki = wv / NS;
  const int r = lane & 15, g = lane >> 4;
  const int64_t slice = blockIdx.x % slices;
  const int64_t nw0 = slice * S::NSL + ni * S::NWC;  // this wave's first column
  const int k0 = ki * S::KW;                         // this wave's first k
  const int64_t rtiles = (M + 15) / 16;
  const int64_t groups = gridDim.x / slices;
  int64_t t = blockIdx.x / slices;
  // zero the padding columns [K, KP) of both buffers once: tile loads write only k < K
  for (int i = tid; i < 2 * 16 * (S::KP - K); i += 64 * kWaves) {
    const int b = i / (16 * (S::KP - K)), rem = i % (16 * (S::KP - K));
    sX[b][rem / (S::KP - K)][K + rem % (S::KP - K)] = 0.0f;
  }
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
  if (t >= rtiles) return;  // uniform over the workgroup: no barrier is skipped by part of it
  // a tile's X rows are one contiguous span of rows * K floats, 16-byte aligned (16 K * 4 B
  // per tile, X aligned); thread tid stages float4s tid, tid + 256, ... of it
  const float invK = 1.0f / static_cast<float>(K);
  float4 st[S::NJ];
  auto load_tile = [&](int64_t tt) {
    const int64_t base = tt * 16 * static_cast<int64_t>(K);
    const int64_t avail = std::min<int64_t>(16, M - tt * 16) * K;  // floats in this tile
#pragma unroll
    for (int j = 0; j < S::NJ; ++j) {
      const int64_t e = 4 * static_cast<int64_t>(tid + 256 * j);
      if (e + 3 < avail) {
        st[j] = *reinterpret_cast<const float4*>(X + base + e);
      } else {
        st[j].x = e < avail ? X[base + e] : 0.0f;
        st[j].y = e + 1 < avail ? X[base + e + 1] : 0.0f;
        st[j].z = e + 2 < avail ? X[base + e + 2] : 0.0f;
        st[j].w = 0.0f;
      }
    }
  };
  auto store_tile = [&](int b) {
#pragma unroll
    for (int j = 0; j < S::NJ; ++j) {
      const int e = 4 * (tid + 256 * j);
      if (e >= 16 * K) break;
      // row of element e: e / K through the reciprocal (exact: e + 0.5 is at least 0.5 / K
      // away from a multiple of K, far above the rounding error at e < 2^14)
      int row = static_cast<int>((static_cast<float>(e) + 0.5f) * invK);
      int col = e - row * K;
      const float v[4] = {st[j].x, st[j].y, st[j].z, st[j].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (row < 16) sX[b][row][col] = v[i];
        if (++col == K) {
          col = 0;
          ++row;
        }
      }
    }
  };
  load_tile(t);
  store_tile(0);
  __syncthreads();
  int cur = 0;
  for (; t < rtiles; t += groups) {
    const bool more = t + groups < rtiles;
    if (more) load_tile(t + groups);  // in flight during this tile's MFMAs
    f4v acc[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[c] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const f4v xa = *reinterpret_cast<const f4v*>(&sX[cur][r][k0 + 16 * q + 4 * g]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[q][s][c], xa[s], acc[c], 0, 0, 0);
    }
    if constexpr (S::KS > 1) {
      if (ki > 0) {
#pragma unroll
        for (int c = 0; c < CB; ++c) sRed[(ki - 1) * NS + ni][c][lane] = acc[c];
      }
      __syncthreads();
      if (ki == 0) {
#pragma unroll
        for (int j = 1; j < S::KS; ++j)
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[c] += sRed[(j - 1) * NS + ni][c][lane];
      }
    }
    const int64_t row = t * 16 + r;
    if (ki == 0 && row < M) {
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int64_t n = nw0 + 16 * c + 4 * g;
        float* y = Y + row * N + n;
        float o[4] = {acc[c][0], acc[c][1], acc[c][2], acc[c][3]};
        if (bias != nullptr) {  // L1-resident; read here instead of holding 4 CB registers
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] += n + j < N ? bias[n + j] : 0.0f;
        }
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
    if (more) store_tile(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
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
    {4, 4, 1},   // K <= 256, N <= 64   (R-GCN dX: 256 -> 64)
    {8, 4, 1},   // K <= 512, N <= 64
    {10, 4, 1},  // K <= 640, N <= 64   (GATConv 602 -> 8 x 8 on Reddit)
};
constexpr int kNumTileCfgs = sizeof(kTileCfgs) / sizeof(kTileCfgs[0]);

// the instance with the least padded MFMA work for (K, N) (X re-reads of extra column
// slices priced at 10 % each); -1: none (K > 640)
int pick_tile(int64_t K, int64_t N) {
  int best = -1;
  double best_cost = 0.0;
  for (int i = 0; i < kNumTileCfgs; ++i) {
    const TileCfg& c = kTileCfgs[i];
    if (K > c.kp()) continue;
    const int64_t slices = (N + c.nsl() - 1) / c.nsl();
    const double cost = static_cast<double>(c.kp()) * slices * c.nsl() * (1.0 + 0.1 * (slices - 1));
    if (best < 0 || cost < best_cost) {
      best = i;
      best_cost = cost;
    }
  }
  return best;
}

template <int KB, int CB, int NS>
void launch_tile(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn, int64_t N,
                 const float* bias, float* Y, hipStream_t s) {
  using S = TileShape<KB, CB, NS>;
  // two workgroups per CU where the W fragment leaves room (<= 256 VGPRs per lane)
  constexpr int OCC = 4 * KB * CB <= 64 ? 2 : 1;
  const int64_t slices = (N + S::NSL - 1) / S::NSL;
  const int64_t rtiles = (M + 15) / 16;
  int64_t groups = std::max<int64_t>(1, 256 * OCC / slices);
  groups = std::min<int64_t>(groups, rtiles);
  hipLaunchKernelGGL((k_project_tile<KB, CB, NS, OCC>), dim3(static_cast<unsigned>(groups * slices)),
                     dim3(64 * kWaves), 0, s, X, M, static_cast<int>(K), W, swk, swn, N, bias, Y, slices);
}

// DGLMI_PROJECT_TILE=1 sends the shapes k_project covers to k_project_tile too (A/B)
bool force_tile() {
  static const bool f = [] {
    const char* e = std::getenv("DGLMI_PROJECT_TILE");
    return e != nullptr && e[0] == '1';
  }();
  return f;
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
    case 6: launch_tile<4, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 7: launch_tile<8, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    case 8: launch_tile<10, 4, 1>(X, M, K, W, swk, swn, N, bias, Y, s); break;
    default: break;  // unsupported: the C entry checks project_supported first
  }
}

}  // namespace dglmi
