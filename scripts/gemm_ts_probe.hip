// Tall-skinny fp32 GEMM on v_mfma_f32_16x16x4_f32 (C = A B, A: M x K row-major, B: K x N
// with strides, K and N small): one wave owns 16 rows x 64 columns, keeps its 64 columns
// of B in registers for the whole launch (persistent), and streams A rows as float4 --
// the k order inside each 16-k block is permuted (lane group g takes k = 4g + s at step
// s) so one lane's four A values are contiguous.  The shape of GraphConv's projection on
// C2 (169 343 x 128 -> 128).  Build: hipcc --offload-arch=gfx950 -O3 -o gemm_ts_probe
// gemm_ts_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// WG = 4 waves sharing one 64-column slice of B, staged once through LDS (coalesced
// rows of W), then each lane copies its 128 fragments LDS -> registers.
template <int K, int NW>
__global__ void __launch_bounds__(256) gemm_ts(const float* __restrict__ A, const float* __restrict__ B,
                                               int64_t sbk, int64_t sbn, float* __restrict__ C,
                                               int64_t M, int64_t N) {
  constexpr int KB = K / 16;   // 16-k blocks
  constexpr int CB = NW / 16;  // 16-column blocks per wave
  __shared__ float sB[K][NW + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t halves = N / NW;
  const int64_t rtiles = (M + 15) / 16;
  const int64_t half = blockIdx.x % halves;
  const int64_t n0 = half * NW;
  // stage B[:, n0 : n0 + NW] (generic strides; coalesced when sbk == 1 by walking k fastest)
  for (int i = threadIdx.x; i < K * NW; i += 256) {
    int k, n;
    if (sbk == 1) { k = i % K; n = i / K; } else { n = i % NW; k = i / NW; }
    sB[k][n] = B[k * sbk + (n0 + n) * sbn];
  }
  __syncthreads();
  float b[KB][4][CB];
#pragma unroll
  for (int q = 0; q < KB; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < CB; ++c) b[q][s][c] = sB[16 * q + 4 * g + s][16 * c + r];
  // row tiles of this slice: wave w of block j takes tiles (j / halves) * 4 + w, + stride
  const int64_t groups = gridDim.x / halves;  // blocks per slice
  const int64_t step = groups * 4;
  int64_t t = (blockIdx.x / halves) * 4 + wv;
  if (blockIdx.x >= groups * halves || t >= rtiles) return;
  auto load_a = [&](int64_t tt, float4 (&a)[KB]) {
    const int64_t row = tt * 16 + r;
#pragma unroll
    for (int q = 0; q < KB; ++q)
      a[q] = row < M ? *reinterpret_cast<const float4*>(A + row * K + 16 * q + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float4 a[KB], an[KB], an2[KB];
  load_a(t, a);
  if (t + step < rtiles) load_a(t + step, an);
  for (; t < rtiles; t += step) {
    const int64_t tn = t + 2 * step;  // two tiles ahead
    if (tn < rtiles) load_a(tn, an2);
    f4 acc[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[c] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const float av[4] = {a[q].x, a[q].y, a[q].z, a[q].w};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        // B as the MFMA's A operand: the result is C's transpose, so lane (r, g) ends
        // with C[row r][16c + 4g .. +3] -- one float4 store per column block
        for (int c = 0; c < CB; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[q][s][c], av[s], acc[c], 0, 0, 0);
    }
    const int64_t row = t * 16 + r;
    if (row < M) {
#pragma unroll
      for (int c = 0; c < CB; ++c)
        *reinterpret_cast<float4*>(C + row * N + n0 + 16 * c + 4 * g) =
            make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
    }
#pragma unroll
    for (int q = 0; q < KB; ++q) { a[q] = an[q]; an[q] = an2[q]; }
  }
}

int main() {
  const int64_t M = 169343, K = 128, N = 128;
  std::vector<float> hA(M * K), hW(N * K);
  std::mt19937 rng(3);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : hA) x = U(rng);
  for (auto& x : hW) x = U(rng);
  float *A, *W, *C;
  CHECK(hipMalloc(&A, M * K * 4));
  CHECK(hipMalloc(&W, N * K * 4));
  CHECK(hipMalloc(&C, M * N * 4));
  CHECK(hipMemcpy(A, hA.data(), M * K * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(W, hW.data(), N * K * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // B = W^T (K x N): B[k][n] = W[n][k] -> strides (1, K), as nn.Linear's weight.t()
  for (int waves : {1024, 1536, 2048}) {
    float best = 1e9f;
    for (int it = 0; it < 8; ++it) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((gemm_ts<128, 64>), dim3(waves / 4), dim3(256), 0, 0, A, W, int64_t{1}, K, C, M, N);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) best = std::min(best, ms);
    }
    std::vector<float> hC(M * N);
    CHECK(hipMemcpy(hC.data(), C, M * N * 4, hipMemcpyDeviceToHost));
    double worst = 0.0;
    for (int64_t i = 0; i < M; i += 997)
      for (int64_t n = 0; n < N; ++n) {
        double ref = 0.0, mag = 0.0;
        for (int64_t k = 0; k < K; ++k) {
          ref += (double)hA[i * K + k] * hW[n * K + k];
          mag += std::fabs((double)hA[i * K + k] * hW[n * K + k]);
        }
        worst = std::max(worst, std::fabs(hC[i * N + n] - ref) / (mag + 1e-30));
      }
    const double flop = 2.0 * M * K * N, bytes = 4.0 * (M * K + M * N);
    std::printf("{\"waves\": %d, \"best_ms\": %.4f, \"TFLOPs\": %.1f, \"GBps\": %.0f, \"worst_rel_err\": %.3g}\n",
                waves, best, flop / best / 1e9, bytes / best / 1e6, worst);
  }
  CHECK(hipFree(A));
  CHECK(hipFree(W));
  CHECK(hipFree(C));
  return 0;
}
