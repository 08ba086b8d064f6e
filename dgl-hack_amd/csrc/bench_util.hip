// Measurement utility for bench.py (not on the message-passing path): a float4
// device-to-device copy, the access pattern the HBM stream rate of
// MI355X_MICROARCH.md is quoted on (6.29 TB/s measured for a float4 copy), so the
// bench line can report the rate this box streams at beside the 8 TB/s spec.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dglmi.h"

namespace {

// One 16 KiB tile per workgroup: each lane loads its 4 float4 (strided by the
// workgroup width, so every load instruction is a coalesced 4 KiB) before storing.
__global__ void __launch_bounds__(256) k_stream_copy(const float4* __restrict__ src,
                                                     float4* __restrict__ dst, int64_t n) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 1024 + threadIdx.x;
  if (base + 768 < n) {
    const float4 a = src[base], b = src[base + 256], c = src[base + 512], d = src[base + 768];
    dst[base] = a;
    dst[base + 256] = b;
    dst[base + 512] = c;
    dst[base + 768] = d;
  } else {
    for (int64_t i = base; i < n && i < base + 1024; i += 256) dst[i] = src[i];
  }
}

}  // namespace

extern "C" int DGLMIStreamCopy(const float* src, float* dst, int64_t num_floats, void* stream) {
  if (src == nullptr || dst == nullptr || num_floats < 0 || num_floats % 4 != 0) return -1;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) return -1;
  const int64_t n4 = num_floats / 4;
  if (n4 == 0) return 0;
  const int64_t tiles = (n4 + 1023) / 1024;
  if (tiles > 0x7fffffff) return -1;
  const unsigned grid = static_cast<unsigned>(tiles);
  hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n4);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
