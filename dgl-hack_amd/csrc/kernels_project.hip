// Bracketing projections Y = X W (+ b) for gfx950 on v_mfma_f32_16x16x4_f32, for the
// tall-skinny shapes GraphConv / GATConv / RelGraphConv project node features with
// (M node rows >> K, N <= a few hundred; fp32 like the reference's torch.matmul).
//
// Design: a wave owns 16 rows x 64 columns of Y.  The 64 columns of W it multiplies by
// stay in its registers for the whole (persistent) launch -- staged once per workgroup
// through LDS with coalesced loads -- and it streams its X rows as float4, two tiles
// ahead.  Inside each 16-k block lane group g takes k = 4g + s at MFMA step s, so a
// lane's four X values are one float4; W goes in as the MFMA's A operand, so the
// accumulator is Y's transpose and each lane ends with four consecutive columns of one
// row (one float4 store per 16-column block).  C2 shape (169 343 x 128 -> 128):
// 66.7 us against 111.2 us for torch.matmul(x, w.t()) (hipBLASLt), scripts/gemm_ts_probe.hip.
#include "internal.h"

#include <algorithm>

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

}  // namespace

// N <= 128: X is read once per 64-column slice, so wider outputs re-read it (5 M x 64 ->
// 256: 2.28 ms here against 2.13 ms on hipBLASLt, profiles/r05_mfma_util.json) and stay there
bool project_supported(int64_t K, int64_t N) {
  return (K == 16 || K == 32 || K == 64 || K == 128) && (N == 64 || N == 128);
}

void launch_project(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn,
                    int64_t N, const float* bias, float* Y, hipStream_t s) {
  if (M == 0) return;
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
}

}  // namespace dglmi
