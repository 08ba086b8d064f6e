// Probe: recompute torch.native_dropout's keep mask on the device from (seed, offset,
// launch geometry) under candidate element -> (thread, draw, component) mappings, to find
// the one torch's fused dropout kernel uses on this build (scripts/philox_probe.py).
// Philox4x32-10 as the Random123 paper defines it (the generator torch's ROCm build draws
// through hiprand/rocrand): counter (x, y) = offset / 4 + draw index, (z, w) = the
// thread's subsequence; key = the 64-bit seed; uniform = 2^-32 + v * 2^-32.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// variant 0: vec4 (c = i/4 -> thread c % G, draw c / G, component i % 4)
// variant 1: vec2, a fresh draw every other pass (component (pass % 2) * 2 + i % 2)
// variant 2: vec2, a fresh draw every pass (component i % 2)
// variant 3: unrolled scalar kernel (thread i % G, q = i / G: draw q / 4, component q % 4)
__global__ void k_probe(int64_t n, int64_t G, uint64_t seed, uint64_t offset, float keep, int variant,
                        uint8_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t t, j;
    int comp;
    if (variant == 0) {
      const int64_t c = i / 4;
      t = c % G; j = c / G; comp = static_cast<int>(i % 4);
    } else if (variant == 1) {
      const int64_t c = i / 2, k = c / G;
      t = c % G; j = k / 2; comp = static_cast<int>((k % 2) * 2 + i % 2);
    } else if (variant == 2) {
      const int64_t c = i / 2;
      t = c % G; j = c / G; comp = static_cast<int>(i % 2);
    } else {
      const int64_t q = i / G;
      t = i % G; j = q / 4; comp = static_cast<int>(q % 4);
    }
    const uint64_t ctr = offset / 4 + static_cast<uint64_t>(j);
    const uint4 r = philox10(make_uint4(static_cast<uint32_t>(ctr), static_cast<uint32_t>(ctr >> 32),
                                        static_cast<uint32_t>(t), static_cast<uint32_t>(static_cast<uint64_t>(t) >> 32)),
                             static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
    const uint32_t v = comp == 0 ? r.x : comp == 1 ? r.y : comp == 2 ? r.z : r.w;
    const float u = 2.3283064365386963e-10f + static_cast<float>(v) * 2.3283064365386963e-10f;
    out[i] = u < keep ? 1 : 0;
  }
}

extern "C" int philox_probe(int64_t n, int64_t G, uint64_t seed, uint64_t offset, float keep, int variant,
                            void* out, void* stream) {
  if (n <= 0) return 0;
  const int64_t want = (n + 255) / 256;
  hipLaunchKernelGGL(k_probe, dim3(static_cast<unsigned>(want < 65536 ? want : 65536)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, G, seed, offset, keep, variant,
                     static_cast<uint8_t*>(out));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
