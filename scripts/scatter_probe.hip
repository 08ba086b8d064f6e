// Random 32-B rows: gather (random read, sequential write) against scatter (sequential
// read, random write) over a random permutation of 114.6 M rows -- the C3 edge count with
// 8 heads -- to price writing a per-edge value in another walk's order (GAT composition:
// the attention in out-CSR order for the node-gradient walk).  Build:
// hipcc --offload-arch=gfx950 -O3 -o scatter_probe scatter_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
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

// two lanes per row (one float4 each), as DGLMIGatherRows
__global__ void __launch_bounds__(256) gather(const float4* __restrict__ s, const int32_t* __restrict__ idx,
                                              int64_t n, float4* __restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < 2 * n; q += stride)
    d[q] = s[2 * static_cast<int64_t>(idx[q >> 1]) + (q & 1)];
}
__global__ void __launch_bounds__(256) scatter(const float4* __restrict__ s, const int32_t* __restrict__ idx,
                                               int64_t n, float4* __restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < 2 * n; q += stride)
    d[2 * static_cast<int64_t>(idx[q >> 1]) + (q & 1)] = s[q];
}
__global__ void __launch_bounds__(256) copy(const float4* __restrict__ s, int64_t n, float4* __restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < 2 * n; q += stride) d[q] = s[q];
}

int main() {
  const int64_t n = 114615892;
  std::vector<int32_t> h(n);
  std::iota(h.begin(), h.end(), 0);
  std::mt19937 rng(1);
  std::shuffle(h.begin(), h.end(), rng);
  float4 *a, *b;
  int32_t* idx;
  CHECK(hipMalloc(&a, n * 32));
  CHECK(hipMalloc(&b, n * 32));
  CHECK(hipMalloc(&idx, n * 4));
  CHECK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(a, 0, n * 32));
  const dim3 grid(65536), blk(256);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[3] = {"copy", "gather", "scatter"};
  for (int k = 0; k < 3; ++k) {
    float best = 1e9f;
    for (int it = 0; it < 6; ++it) {
      CHECK(hipEventRecord(e0));
      if (k == 0) hipLaunchKernelGGL(copy, grid, blk, 0, 0, a, n, b);
      else if (k == 1) hipLaunchKernelGGL(gather, grid, blk, 0, 0, a, idx, n, b);
      else hipLaunchKernelGGL(scatter, grid, blk, 0, 0, a, idx, n, b);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) best = std::min(best, ms);
    }
    std::printf("{\"kernel\": \"%s\", \"rows\": %lld, \"row_bytes\": 32, \"best_ms\": %.4f}\n", names[k],
                static_cast<long long>(n), best);
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(idx));
  return 0;
}
