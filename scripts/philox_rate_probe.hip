// Throughput of the Philox4x32-10 round's two 32x32 -> 64 multiplies on gfx950:
// v_mul_hi_u32 + v_mul_lo_u32 (what hipcc emits) against one v_mad_u64_u32 each.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/philox_rate_probe.hip -o scripts/philox_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ void mul2(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  hi = __umulhi(a, b);
  lo = a * b;
}
__device__ __forceinline__ void mad2(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t r, c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(c) : "v"(a), "v"(b));
  hi = static_cast<uint32_t>(r >> 32);
  lo = static_cast<uint32_t>(r);
}
template <bool MAD>
__global__ void k(uint32_t* out, int reps, uint32_t m0, uint32_t m1) {
  uint32_t x = threadIdx.x, y = blockIdx.x, z = x ^ 0x1234u, w = y + 7u, k0 = 1u, k1 = 2u;
  for (int i = 0; i < reps; ++i) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      uint32_t h0, l0, h1, l1;
      if (MAD) { mad2(m0, x, h0, l0); mad2(m1, z, h1, l1); }
      else { mul2(m0, x, h0, l0); mul2(m1, z, h1, l1); }
      const uint32_t nx = h1 ^ y ^ k0, nz = h0 ^ w ^ k1;
      y = l1; w = l0; x = nx; z = nz;
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y ^ z ^ w;
}
int main() {
  uint32_t* out;
  hipMalloc(&out, 8192 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int reps = 200;
  for (int mad = 0; mad < 2; ++mad) {
    for (int t = 0; t < 3; ++t) {
      hipEventRecord(a);
      if (mad) hipLaunchKernelGGL(k<true>, dim3(8192), dim3(256), 0, 0, out, reps, 0xD2511F53u, 0xCD9E8D57u);
      else hipLaunchKernelGGL(k<false>, dim3(8192), dim3(256), 0, 0, out, reps, 0xD2511F53u, 0xCD9E8D57u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double blocks = 8192.0 * 256 * reps;
      printf("{\"mad_u64\": %d, \"ms\": %.3f, \"G_philox_blocks_per_s\": %.1f}\n", mad, ms, blocks / ms / 1e6);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
