// Variants of the float4 stream copy bench.py reports beside the 8 TB/s spec
// (DGLMIStreamCopy, csrc/bench_util.hip): read + write bytes / time for a 4 GiB
// fp32 buffer.  Build: hipcc --offload-arch=gfx950 -O3 -o stream_copy_probe
// stream_copy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

// V0: one 16 KiB tile per workgroup (the shipped form)
__global__ void __launch_bounds__(256) v0(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 1024 + threadIdx.x;
  if (b + 768 < n) {
    float4 x0 = s[b], x1 = s[b + 256], x2 = s[b + 512], x3 = s[b + 768];
    d[b] = x0; d[b + 256] = x1; d[b + 512] = x2; d[b + 768] = x3;
  } else {
    for (int64_t i = b; i < n && i < b + 1024; i += 256) d[i] = s[i];
  }
}

// V1: 32 KiB tile per workgroup (8 float4 per lane in flight)
__global__ void __launch_bounds__(256) v1(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 2048 + threadIdx.x;
  if (b + 1792 < n) {
    float4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = s[b + 256 * k];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[b + 256 * k] = x[k];
  } else {
    for (int64_t i = b; i < n && i < b + 2048; i += 256) d[i] = s[i];
  }
}

typedef float v4f __attribute__((ext_vector_type(4)));

// V2: V0 with non-temporal loads and stores
__global__ void __launch_bounds__(256) v2(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 1024 + threadIdx.x;
  if (b + 768 < n) {
    const v4f* sv = reinterpret_cast<const v4f*>(s);
    v4f* dv = reinterpret_cast<v4f*>(d);
    v4f x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = __builtin_nontemporal_load(sv + b + 256 * k);
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(x[k], dv + b + 256 * k);
  } else {
    for (int64_t i = b; i < n && i < b + 1024; i += 256) d[i] = s[i];
  }
}

// V3: V0 with plain loads, non-temporal stores
__global__ void __launch_bounds__(256) v3(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 1024 + threadIdx.x;
  if (b + 768 < n) {
    const v4f* sv = reinterpret_cast<const v4f*>(s);
    v4f* dv = reinterpret_cast<v4f*>(d);
    v4f x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = sv[b + 256 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(x[k], dv + b + 256 * k);
  } else {
    for (int64_t i = b; i < n && i < b + 1024; i += 256) d[i] = s[i];
  }
}

// V4: persistent grid-stride, 8 waves per CU resident, 4 float4 per lane per trip
__global__ void __launch_bounds__(256) v4(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t tiles = n / 1024;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t b = t * 1024 + threadIdx.x;
    float4 x0 = s[b], x1 = s[b + 256], x2 = s[b + 512], x3 = s[b + 768];
    d[b] = x0; d[b + 256] = x1; d[b + 512] = x2; d[b + 768] = x3;
  }
  if (blockIdx.x == 0)
    for (int64_t i = tiles * 1024 + threadIdx.x; i < n; i += 256) d[i] = s[i];
}

// V5: 512-thread workgroups, 4 float4 per lane (32 KiB per workgroup)
__global__ void __launch_bounds__(512) v5(const float4* __restrict__ s, float4* __restrict__ d, int64_t n) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 2048 + threadIdx.x;
  if (b + 1536 < n) {
    float4 x0 = s[b], x1 = s[b + 512], x2 = s[b + 1024], x3 = s[b + 1536];
    d[b] = x0; d[b + 512] = x1; d[b + 1024] = x2; d[b + 1536] = x3;
  } else {
    for (int64_t i = b; i < n && i < b + 2048; i += 512) d[i] = s[i];
  }
}

int main() {
  const int64_t bytes = int64_t(4) << 30;
  const int64_t n = bytes / 16;
  float4 *s, *d;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMemset(s, 1, bytes));
  CHECK(hipMemset(d, 0, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"v0_16KiB_tile", "v1_32KiB_tile", "v2_nt_load_store", "v3_nt_store",
                         "v4_persistent_2048wg", "v5_512thr_32KiB"};
  for (int v = 0; v < 6; ++v) {
    auto launch = [&]() {
      switch (v) {
        case 0: hipLaunchKernelGGL(v0, dim3((n + 1023) / 1024), dim3(256), 0, 0, s, d, n); break;
        case 1: hipLaunchKernelGGL(v1, dim3((n + 2047) / 2048), dim3(256), 0, 0, s, d, n); break;
        case 2: hipLaunchKernelGGL(v2, dim3((n + 1023) / 1024), dim3(256), 0, 0, s, d, n); break;
        case 3: hipLaunchKernelGGL(v3, dim3((n + 1023) / 1024), dim3(256), 0, 0, s, d, n); break;
        case 4: hipLaunchKernelGGL(v4, dim3(2048), dim3(256), 0, 0, s, d, n); break;
        case 5: hipLaunchKernelGGL(v5, dim3((n + 2047) / 2048), dim3(512), 0, 0, s, d, n); break;
      }
    };
    for (int w = 0; w < 3; ++w) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double tbs = 2.0 * bytes * reps / (ms * 1e-3) / 1e12;
    std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", names[v], ms / reps, tbs);
  }
  CHECK(hipFree(s));
  CHECK(hipFree(d));
  return 0;
}
