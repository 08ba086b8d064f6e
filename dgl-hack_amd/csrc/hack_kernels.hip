// Helpers of the C entries that replace the hack's R-GCN PackedFuncs
// (_CAPI_DGLRgcnLayer0/1[Backward], binary_reduce.cc:411-450): relation-expanded
// column ids, the relation-weight layout change, and an LDS-tiled fp32-input MFMA
// GEMM for the (N x K) . (K x R*F) transforms.
//
// The hack computes one (F_in x F_out) product PER EDGE inside its gather
// (binary_reduce_impl.cu:1050-1117).  Here, as on the Python path
// (dgl/backend.py rgcn_layer1), the relation transforms are ONE dense product
// over the node rows and the edges only gather: y[u * R + t] rows, summed by the
// load-balanced reduce.  The Python path runs that product on hipBLASLt (torch);
// the C entries keep the library free of a second BLAS runtime in the caller's
// process and use the kernel below -- these shapes (K, F <= a few hundred) are
// bound by reading X and writing Y, not by the FMAs.
#include "internal.h"

namespace dglmi {
namespace {

constexpr int kBlock = 256;

// relation-expanded ids: mode 0: etype * mul + id (type-major), 1: id * mul + etype
__global__ void k_typed_ids(const int32_t* __restrict__ ids, const int32_t* __restrict__ eids,
                            const int32_t* __restrict__ etypes, int64_t nnz, int64_t mul, int mode,
                            int32_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < nnz; p += stride) {
    const int64_t t = etypes[eids ? eids[p] : p];
    const int64_t id = ids[p];
    out[p] = static_cast<int32_t>(mode == 0 ? t * mul + id : id * mul + t);
  }
}

// to_cat: out[k, r*X + x] = w[r, k, x]; else out[r, k, x] = w[k, r*X + x]
__global__ void k_permute_rkx(const float* __restrict__ w, int64_t R, int64_t K, int64_t X,
                              bool to_cat, float* __restrict__ out) {
  const int64_t n = R * K * X;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t x = i % X, k = (i / X) % K, r = i / (X * K);  // i = (r, k, x)
    const int64_t j = k * R * X + r * X + x;                      // (k, r*X + x)
    if (to_cat) out[j] = w[i];
    else out[i] = w[j];
  }
}

// C[z] (M x N, row-major) = sum over k in split z of A[m, k] * B[k, n]; A and B by
// (row, col) strides.  fp32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32, an
// fmaf chain per output): a 128 x 64 output tile per workgroup, each of the four
// waves owning 32 rows x 64 columns (two 32 x 32 accumulators); 32-deep slices of
// A and B staged in LDS with loads that run along each operand's unit-stride
// dimension.
using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int kTM = 128, kTN = 64, kTK = 32;

__global__ void __launch_bounds__(kBlock) k_gemm(const float* __restrict__ A, int64_t a_rs,
                                                 int64_t a_cs, const float* __restrict__ B,
                                                 int64_t b_rs, int64_t b_cs, float* __restrict__ C,
                                                 int64_t M, int64_t N, int64_t K, int64_t k_split) {
  __shared__ float As[kTM][kTK + 1];
  __shared__ float Bs[kTK][kTN + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // 1-D grid, column tiles fastest: the blocks that share an A row slice run
  // back to back, so the slice is read from HBM once and from L2 after that
  const int64_t n_tiles = (N + kTN - 1) / kTN;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) / n_tiles * kTM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x) % n_tiles * kTN;
  const int64_t kb = static_cast<int64_t>(blockIdx.z) * k_split;
  const int64_t ke = kb + k_split < K ? kb + k_split : K;
  f32x16 acc0 = {}, acc1 = {};
  for (int64_t k0 = kb; k0 < ke; k0 += kTK) {
    for (int i = threadIdx.x; i < kTM * kTK; i += kBlock) {
      const int kk = a_cs == 1 ? i % kTK : i / kTM;
      const int mm = a_cs == 1 ? i / kTK : i % kTM;
      const int64_t m = m0 + mm, k = k0 + kk;
      As[mm][kk] = (m < M && k < ke) ? A[m * a_rs + k * a_cs] : 0.0f;
    }
    for (int i = threadIdx.x; i < kTK * kTN; i += kBlock) {
      const int kk = b_cs == 1 ? i / kTN : i % kTK;
      const int nn = b_cs == 1 ? i % kTN : i / kTK;
      const int64_t n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < N && k < ke) ? B[k * b_rs + n * b_cs] : 0.0f;
    }
    __syncthreads();
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < kTK; kk += 2) {
      const float a = As[w * 32 + r][kk + h];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[kk + h][r], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[kk + h][32 + r], acc1, 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  float* Cz = C + static_cast<int64_t>(blockIdx.z) * M * N;
  const int col = lane & 31;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int64_t m = m0 + w * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (m >= M) continue;
    const int64_t n = n0 + col;
    if (n < N) Cz[m * N + n] = acc0[reg];
    if (n + 32 < N) Cz[m * N + n + 32] = acc1[reg];
  }
}

// out[i] = sum over z (in order) of parts[z * n + i]
__global__ void k_sum_splits(const float* __restrict__ parts, int splits, int64_t n,
                             float* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = 0.0f;
    for (int z = 0; z < splits; ++z) s += parts[z * n + i];
    out[i] = s;
  }
}

unsigned grid1(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

void launch_typed_ids(const int32_t* ids, const int32_t* eids, const int32_t* etypes, int64_t nnz,
                      int64_t mul, int mode, int32_t* out, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_typed_ids, dim3(grid1(nnz)), dim3(kBlock), 0, s, ids, eids, etypes, nnz, mul,
                     mode, out);
}

void launch_permute_rkx(const float* w, int64_t R, int64_t K, int64_t X, bool to_cat, float* out,
                        hipStream_t s) {
  if (R * K * X <= 0) return;
  hipLaunchKernelGGL(k_permute_rkx, dim3(grid1(R * K * X)), dim3(kBlock), 0, s, w, R, K, X, to_cat,
                     out);
}

int64_t gemm_splits(int64_t M, int64_t N, int64_t K) {
  // split the reduction when the output has too few tiles to fill 256 CUs
  const int64_t tiles = ((M + kTM - 1) / kTM) * ((N + kTN - 1) / kTN);
  int64_t splits = 1;
  while (tiles * splits < 4096 && K / (splits * 2) >= 512 && splits < 2048) splits *= 2;
  return splits;
}

void launch_gemm(const float* A, int64_t a_rs, int64_t a_cs, const float* B, int64_t b_rs,
                 int64_t b_cs, float* C, int64_t M, int64_t N, int64_t K, int64_t splits,
                 float* partials, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  if (K <= 0) {
    launch_fill(C, M * N, 0.0f, s);
    return;
  }
  const int64_t k_split = ((K + splits - 1) / splits + kTK - 1) / kTK * kTK;
  const int64_t used = (K + k_split - 1) / k_split;
  const dim3 grid(static_cast<unsigned>(((M + kTM - 1) / kTM) * ((N + kTN - 1) / kTN)), 1,
                  static_cast<unsigned>(used));
  if (used == 1) {
    hipLaunchKernelGGL(k_gemm, grid, dim3(kBlock), 0, s, A, a_rs, a_cs, B, b_rs, b_cs, C, M, N, K,
                       k_split);
    return;
  }
  hipLaunchKernelGGL(k_gemm, grid, dim3(kBlock), 0, s, A, a_rs, a_cs, B, b_rs, b_cs, partials, M, N,
                     K, k_split);
  hipLaunchKernelGGL(k_sum_splits, dim3(grid1(M * N)), dim3(kBlock), 0, s, partials,
                     static_cast<int>(used), M * N, C);
}

}  // namespace dglmi
