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
#include <cstdlib>
#include <stdexcept>

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

// ---------------------------------------------------------------------------
// Tall-skinny products of the R-GCN entries: one dimension is the node count (10^6 -
// 10^7 rows), the other two are <= 256.  k_gemm above moves the same bytes 2-5x slower
// on these shapes (C5, 5 M x 64 -> 256: 4.0 ms, 256 -> 64: 3.7 ms, the 5 M-row
// reduction 6.95 ms; scripts/rgcn_capi_probe.py under rocprofv3), so each shape gets
// its own kernel (v_mfma_f32_32x32x2_f32, exact f32 like k_gemm):
//  * k_gemm_rows: C (M x N) = A (M x K) . B (K x N), A and C row-major.  All of B sits
//    in LDS for the block's life; each of the 8 waves owns 32-row tiles of C (strided
//    over the grid), stages its A tile through a private LDS slice 32 columns at a time
//    (the next slice is loaded into registers while the MFMAs run on this one, so the
//    waves need no block barrier) and writes C once, non-temporally.
//  * k_gemm_tn: C (M x N) = A^T . B, A (R x M) and B (R x N) row-major, R = the node
//    count: every block reduces a contiguous range of rows into its own M x N partial
//    (32-row slices of A and B staged through two LDS buffers), k_sum_splits adds the
//    partials in block order (deterministic).
constexpr int kGemmThreads = 512;  // 8 waves, one block per CU (LDS)
constexpr int kSlice = 32;
// LDS row stride (floats) for rows of `cols` floats read as MFMA operands: lanes r and
// r + 32 read rows kk and kk + 1, so a stride == 32 (mod 64) puts them in different
// bank halves
__host__ __device__ constexpr int mfma_lds_stride(int cols) {
  return (cols % 64 == 0) ? cols + 32 : cols;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// NB = N / 32 (rounded up), KP = K rounded up to kSlice; needs K % 4 == 0, lda % 4 == 0
// and a 16-byte aligned A (the host checks).
template <int NB, int KP>
__global__ void __launch_bounds__(kGemmThreads) k_gemm_rows(const float* __restrict__ A,
                                                        int64_t lda, const float* __restrict__ B,
                                                        int64_t b_rs, int64_t b_cs,
                                                        float* __restrict__ C, int64_t M, int N,
                                                        int K) {
  constexpr int SB = mfma_lds_stride(NB * 32);
  constexpr int SA = kSlice + 1;
  constexpr int NSL = KP / kSlice;
  __shared__ float Bs[KP * SB];
  __shared__ float As[8][32 * SA];
  for (int i = threadIdx.x; i < KP * NB * 32; i += kGemmThreads) {
    const int k = i / (NB * 32), n = i % (NB * 32);
    Bs[k * SB + n] = (k < K && n < N) ? B[k * b_rs + n * b_cs] : 0.0f;
  }
  __syncthreads();  // the only block barrier: the waves run independently after it
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  float* as = As[w];
  const int64_t tiles = (M + 31) / 32;
  const int64_t step = static_cast<int64_t>(gridDim.x) * 8;
  int64_t tile = static_cast<int64_t>(blockIdx.x) * 8 + w;
  if (tile >= tiles) return;
  // staging map: lane -> rows (lane >> 3) + 8 j of the tile, float4 column lane & 7
  const int srow = lane >> 3, sc4 = lane & 7;
  float4 v[4];
  auto load = [&](int64_t t, int sl) {
    const int k = sl * kSlice + 4 * sc4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = t * 32 + srow + 8 * j;
      v[j] = (m < M && k < K) ? *reinterpret_cast<const float4*>(A + m * lda + k)
                              : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  };
  load(tile, 0);
  while (true) {
    f32x16 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
      wave_lds_sync();  // every lane is done reading the previous slice
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float* d = as + (srow + 8 * j) * SA + 4 * sc4;
        d[0] = v[j].x;
        d[1] = v[j].y;
        d[2] = v[j].z;
        d[3] = v[j].w;
      }
      wave_lds_sync();
      // the next slice (or the next tile's first) is in flight during the MFMAs
      if (sl + 1 < NSL) load(tile, sl + 1);
      else if (tile + step < tiles) load(tile + step, 0);
#pragma unroll
      for (int kk = 0; kk < kSlice; kk += 2) {
        const float a = as[r * SA + kk + h];
        const float* brow = Bs + (sl * kSlice + kk + h) * SB + r;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, brow[nb * 32], acc[nb], 0, 0, 0);
      }
    }
    // C/D map: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int64_t m = tile * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (m >= M) continue;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = nb * 32 + r;
        if (n < N) __builtin_nontemporal_store(acc[nb][reg], C + m * N + n);
      }
    }
    tile += step;
    if (tile >= tiles) break;
  }
}

// C partial of block z (M x N) = sum over rows q in [z * rows_per_block, ...) of
// A[q, m] * B[q, n].  MB = M / 32, NB = N / 32 (rounded up), MB * NB <= 16: wave w owns
// the (m, n) 32 x 32 blocks w and w + 8.  Needs M, N, lda, ldb % 4 == 0 and 16-byte
// aligned A, B.
template <int MB, int NB>
// at most 2 waves per SIMD (one block per CU): the two register sets of staged slices
// then fit without spills at every instance
__global__ void __launch_bounds__(kGemmThreads) __attribute__((amdgpu_waves_per_eu(1, 2)))
k_gemm_tn(const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ parts, int64_t R, int M,
                                                      int N, int64_t rows_per_block) {
  constexpr int SA = mfma_lds_stride(MB * 32), SB = mfma_lds_stride(NB * 32);
  constexpr int A4 = MB * 8, B4 = NB * 8;                  // float4 per staged row
  constexpr int AL = (kSlice * A4 + kGemmThreads - 1) / kGemmThreads;
  constexpr int BL = (kSlice * B4 + kGemmThreads - 1) / kGemmThreads;
  constexpr int BPW = (MB * NB + 7) / 8;  // 32 x 32 output blocks per wave
  static_assert(BPW <= 3, "at most three 32 x 32 blocks per wave");
  __shared__ float As[2][kSlice * SA];
  __shared__ float Bs[2][kSlice * SB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < R ? r0 + rows_per_block : R;
  const int nsl = r1 > r0 ? static_cast<int>((r1 - r0 + kSlice - 1) / kSlice) : 0;
  // two slices in flight: the registers of slice sl + 2 are loaded while slice sl is
  // multiplied (one slice ahead left the fabric idle: 2.8 TB/s on the C5 shapes)
  float4 va[2][AL], vb[2][BL];
  auto load = [&](int sl, int rb) {
#pragma unroll
    for (int j = 0; j < AL; ++j) {
      const int idx = threadIdx.x + j * kGemmThreads;
      const int row = idx / A4, c = 4 * (idx % A4);
      const int64_t q = r0 + static_cast<int64_t>(sl) * kSlice + row;
      va[rb][j] = (idx < kSlice * A4 && q < r1 && c < M)
                  ? *reinterpret_cast<const float4*>(A + q * lda + c)
                  : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < BL; ++j) {
      const int idx = threadIdx.x + j * kGemmThreads;
      const int row = idx / B4, c = 4 * (idx % B4);
      const int64_t q = r0 + static_cast<int64_t>(sl) * kSlice + row;
      vb[rb][j] = (idx < kSlice * B4 && q < r1 && c < N)
                  ? *reinterpret_cast<const float4*>(B + q * ldb + c)
                  : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  };
  auto store = [&](int buf, int rb) {
#pragma unroll
    for (int j = 0; j < AL; ++j) {
      const int idx = threadIdx.x + j * kGemmThreads;
      if (idx < kSlice * A4)
        *reinterpret_cast<float4*>(&As[buf][(idx / A4) * SA + 4 * (idx % A4)]) = va[rb][j];
    }
#pragma unroll
    for (int j = 0; j < BL; ++j) {
      const int idx = threadIdx.x + j * kGemmThreads;
      if (idx < kSlice * B4)
        *reinterpret_cast<float4*>(&Bs[buf][(idx / B4) * SB + 4 * (idx % B4)]) = vb[rb][j];
    }
  };
  f32x16 acc[BPW];
#pragma unroll
  for (int i = 0; i < BPW; ++i) acc[i] = f32x16{};
  if (nsl > 0) load(0, 0);
  if (nsl > 1) load(1, 1);
  // slice sl lives in LDS buffer sl & 1 and, until stored, in register set sl & 1
  auto step = [&](int sl, int rb) {
    store(sl & 1, rb);
    __syncthreads();
    if (sl + 2 < nsl) load(sl + 2, rb);
    const float* as = As[sl & 1];
    const float* bs = Bs[sl & 1];
#pragma unroll
    for (int kk = 0; kk < kSlice; kk += 2) {
#pragma unroll
      for (int i = 0; i < BPW; ++i) {
        const int b = w + 8 * i;  // wave-uniform
        if (b < MB * NB)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(as[(kk + h) * SA + (b / NB) * 32 + r],
                                                        bs[(kk + h) * SB + (b % NB) * 32 + r], acc[i],
                                                        0, 0, 0);
      }
    }
  };
  int sl = 0;
  for (; sl + 1 < nsl; sl += 2) {
    step(sl, 0);
    step(sl + 1, 1);
  }
  if (sl < nsl) step(sl, 0);
  float* P = parts + static_cast<int64_t>(blockIdx.x) * M * N;
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int b = w + 8 * i;
    if (b >= MB * NB) continue;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = (b / NB) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, n = (b % NB) * 32 + r;
      if (m < M && n < N) P[m * N + n] = acc[i][reg];
    }
  }
}

// ---------------------------------------------------------------------------
// Fused R-GCN layer 1: aggregate each relation's rows first, transform after, in one
// kernel.  out[v] = sum_t (sum_{e = (u -> v), type t} w_e T[u]) . W_t: every wave owns
// 32-row tiles of out (drawn from a queue); for each relation t it gathers the 32
// rows' relation-t sums of T (64-float rows, 16 lanes per row; the tile's edges cut
// into four equal shares, one per 16-lane group, rows cut by a share boundary
// finished through per-group carries in group order; 8 gathers in flight per lane)
// into its private LDS slot, and one MFMA pass
// (v_mfma_f32_32x32x2_f32) adds slot . W_t into the tile's accumulators; W (all
// relations, <= 64 KB) sits in LDS for the block's life.  No Y = T . W_cat table
// (5.1 GB on C5) is written or gathered: the gathers read T (1.3 GB) and the only HBM
// write is the output.  Walks the relation-major CSR (rows t * num_rows + v, the
// prepared state's in_rel / out_typed[0]), whose rows of one relation and tile are
// contiguous.  With Lw (RelGraphConv's self-loop) one more pass multiplies the tile's
// own rows of T by Lw; BWD also stores those rows as gy's last block, so one GEMM gives
// the relation and self-loop weight gradients.  BWD with out == nullptr (no input
// gradient wanted) skips the MFMA passes and stores only gy.  Deterministic: each row's edges in position order (a cut row's
// share sums added in share order), then relations and k in order.  BWD: the same walk over the relation-major out-CSR gathers
// grad_out rows into G_t (stored to gy for the weight gradient) and adds
// G_t . W_t^T into grad_hidden.  The weights enter as W[t][k][n] =
// W_src[t * ws_t + k * ws_k + n * ws_n] (k over the gathered width 64).
constexpr int kFusedW = 64;  // gathered row width (floats)
constexpr int kSlotStride = kFusedW + 1;
// LDS for the weights: (relations + self-loop) x 64 x (out width rounded to 32)
constexpr int kFusedWsFloats = 20480;
// tile queues of the fused kernels: tiles per atomic, and the spacing of the eight
// counters (unsigned; one 128-B line each)
constexpr int kTileGrab = 2;
constexpr int kCtrStride = 32;

// Lane u of each 16-lane row (DPP row_newbcast; u folds to a constant once unrolled):
// what __shfl(v, u, 16) returns, without the ds_bpermute round trip through the LDS
__device__ __forceinline__ int row_bcast16(int v, int u) {
#if DGLMI_PROBES
  return __shfl(v, u, 16);  // probe build: the round-3 walk (ds_bpermute), for A/B timing
#endif
  switch (u & 15) {
#define DGLMI_RB(U) case U: return __builtin_amdgcn_update_dpp(0, v, 0x150 + U, 0xF, 0xF, false);
    DGLMI_RB(0) DGLMI_RB(1) DGLMI_RB(2) DGLMI_RB(3) DGLMI_RB(4) DGLMI_RB(5) DGLMI_RB(6)
    DGLMI_RB(7) DGLMI_RB(8) DGLMI_RB(9) DGLMI_RB(10) DGLMI_RB(11) DGLMI_RB(12) DGLMI_RB(13)
    DGLMI_RB(14) DGLMI_RB(15)
#undef DGLMI_RB
  }
  return 0;
}

// the slot's rows -> gy[v][t * 64 + c], gy rows `mats` blocks of 64 wide (the weight
// gradients' operand: G_t per relation, then the tile's own rows for the self-loop)
__device__ __forceinline__ void store_gy(const float* slot, float* gy, int64_t v0, int g, int q,
                                         int tile_rows, int mats, int t) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (8 * g + i >= tile_rows) break;
    const float* s = slot + (8 * g + i) * kSlotStride + 4 * q;
    float* d = gy + (v0 + 8 * g + i) * (static_cast<int64_t>(mats) * kFusedW) + t * kFusedW + 4 * q;
    __builtin_nontemporal_store(s[0], d);
    __builtin_nontemporal_store(s[1], d + 1);
    __builtin_nontemporal_store(s[2], d + 2);
    __builtin_nontemporal_store(s[3], d + 3);
  }
}

// acc[nb] += slot (32 x 64) . wt (64 x SW): one v_mfma_f32_32x32x2_f32 per 2 k and
// 32 output columns
template <int NB, int SW>
__device__ __forceinline__ void mfma_slot(const float* slot, const float* wt, int r, int hb,
                                          f32x16 (&acc)[NB]) {
#pragma unroll
  for (int kk = 0; kk < kFusedW; kk += 2) {
    const float a = slot[r * kSlotStride + kk + hb];
    const float* brow = wt + (kk + hb) * SW + r;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      acc[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, brow[nb * 32], acc[nb], 0, 0, 0);
  }
}

template <bool BWD, int NB>
__global__ void __launch_bounds__(kGemmThreads) k_rgcn_fused(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ cols,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ eids, const float* __restrict__ w,
    const float* __restrict__ T, const float* __restrict__ W, int64_t ws_t, int64_t ws_k,
    int64_t ws_n, float* __restrict__ out, float* __restrict__ gy, int64_t num_rows, int R,
    int out_w, const float* __restrict__ bias, const float* __restrict__ addend,
    const float* __restrict__ Lw, unsigned* __restrict__ tile_ctr) {
  constexpr int SW = NB * 32;
  __shared__ float Ws[kFusedWsFloats];
  __shared__ float slots[8][32 * kSlotStride];
  __shared__ float carries[8][4][kFusedW];
  const int RL = R + (Lw != nullptr);  // the self-loop weight is one more matrix
  for (int i = threadIdx.x; i < RL * kFusedW * SW; i += kGemmThreads) {
    const int t = i / (kFusedW * SW), k = (i / SW) % kFusedW, n = i % SW;
    Ws[i] = n >= out_w ? 0.0f
                       : (t < R ? W[t * ws_t + k * ws_k + n * ws_n] : Lw[k * ws_k + n * ws_n]);
  }
  __syncthreads();  // the only block barrier
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 31, hb = lane >> 5;
  const int g = lane >> 4, q = lane & 15;  // 16-lane group, float4 column
  float* slot = slots[wv];
  float* carry = carries[wv][0];
  const int64_t tiles = (num_rows + 31) / 32;
  // tiles from queues (one vector atomic per kTileGrab tiles): a wave that drew a hub
  // row's tile does not hold the others back, and a tile's result does not depend on
  // which wave computed it.  Eight queues (fewer on a grid of fewer blocks), tiles q,
  // q + 8, ... in queue q, served by the blocks b with b % 8 == q (one XCD each under
  // round-robin dispatch; correctness does not depend on the placement): the atomics
  // of one counter serialise, and a single counter for every wave cost ~10 ns per
  // tile, 1.6 ms of a C5 launch.
  // (fewer queues than blocks on a small grid: every queue must have a server)
  const int nq = gridDim.x < 8 ? static_cast<int>(gridDim.x) : 8;
  const int64_t qid = blockIdx.x % nq;
  unsigned* ctr = tile_ctr + qid * kCtrStride;
  const int64_t qtiles = tiles > qid ? (tiles - qid + nq - 1) / nq : 0;
  for (int64_t k0 = 0;;) {
    if ((k0 & (kTileGrab - 1)) == 0) {
      unsigned tv = 0;
      if (lane == 0) tv = atomicAdd(ctr, static_cast<unsigned>(kTileGrab));
      k0 = static_cast<unsigned>(__shfl(static_cast<int>(tv), 0));
    }
    if (k0 >= qtiles) break;
    const int64_t tile = qid + nq * k0;
    ++k0;
    const int64_t v0 = tile * 32;
    const int tile_rows = num_rows - v0 < 32 ? static_cast<int>(num_rows - v0) : 32;
    f32x16 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
    for (int t = 0; t < RL; ++t) {
      if (t == R) {
        // self-loop: the tile's own rows of T (coalesced, no gather) through Lw
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int64_t v = v0 + 8 * g + i;
          const float4 a = v < num_rows
                               ? *reinterpret_cast<const float4*>(T + v * kFusedW + 4 * q)
                               : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          float* d = slot + (8 * g + i) * kSlotStride + 4 * q;
          d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
        }
        wave_lds_sync();
        if constexpr (BWD) store_gy(slot, gy, v0, g, q, tile_rows, RL, t);
        if (out != nullptr) mfma_slot<NB, SW>(slot, Ws + t * kFusedW * SW, r, hb, acc);
        wave_lds_sync();
        continue;
      }
      const int64_t base = static_cast<int64_t>(t) * num_rows + v0;
      const int64_t pb = ptr[base], pe = ptr[base + tile_rows];
      if (!BWD && pb == pe) continue;  // no relation-t edge into the tile
      // zero the 32 slot rows (8 per group; the stores below come later in this
      // wave's program order)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float* d = slot + (8 * g + i) * kSlotStride + 4 * q;
        d[0] = d[1] = d[2] = d[3] = 0.0f;
      }
      // the tile's relation-t edges (contiguous) in four equal shares, one per
      // 16-lane group; a row cut by a share boundary is stored by the group holding
      // its first edge and continued in the next groups' carries
      const int64_t share = (pe - pb + 3) / 4;
      const int64_t gb = pb + g * share < pe ? pb + g * share : pe;
      const int64_t ge = gb + share < pe ? gb + share : pe;
      const bool cont = gb < ge && gb > pb && rows[gb - 1] == rows[gb];
      bool first = true;
      int crow = -1;  // the row this group's carry continues (-1: none)
      float4 a4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      int cur = -1;
      auto flush = [&]() {
        float* d = (first && cont) ? carry + g * kFusedW + 4 * q
                                   : slot + cur * kSlotStride + 4 * q;
        if (first && cont) crow = cur;
        d[0] = a4.x; d[1] = a4.y; d[2] = a4.z; d[3] = a4.w;
        first = false;
      };
      for (int64_t p = gb; p < ge; p += 16) {
        const int n = ge - p < 16 ? static_cast<int>(ge - p) : 16;
        int my_col = 0, my_row = -1;
        float my_w = 0.0f;
        if (q < n) {
          my_col = cols[p + q];
          my_row = static_cast<int>(rows[p + q] - base);
          my_w = w[eids ? eids[p + q] : p + q];
        }
#pragma unroll
        for (int j0 = 0; j0 < 16; j0 += 8) {
          float4 x[8];
          float wj[8];
          int rj[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            // the group's edge j0 + u: DPP row broadcasts (VALU, no LDS round trip)
            const int c = row_bcast16(my_col, j0 + u);
            rj[u] = row_bcast16(my_row, j0 + u);
            wj[u] = __int_as_float(row_bcast16(__float_as_int(my_w), j0 + u));
            x[u] = *reinterpret_cast<const float4*>(T + static_cast<int64_t>(c) * kFusedW + 4 * q);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (rj[u] < 0) break;  // past the batch (group-uniform)
            if (rj[u] != cur) {
              if (cur >= 0) flush();
              a4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
              cur = rj[u];
            }
            a4.x += wj[u] * x[u].x;
            a4.y += wj[u] * x[u].y;
            a4.z += wj[u] * x[u].z;
            a4.w += wj[u] * x[u].w;
          }
        }
      }
      if (cur >= 0) flush();
      wave_lds_sync();
      // carries into their rows, in group order (deterministic)
#pragma unroll
      for (int gg = 1; gg < 4; ++gg) {
        const int cr = __shfl(crow, gg * 16);
        if (cr >= 0) slot[cr * kSlotStride + lane] += carry[gg * kFusedW + lane];
      }
      wave_lds_sync();
      if constexpr (BWD) store_gy(slot, gy, v0, g, q, tile_rows, RL, t);
      if (out != nullptr) mfma_slot<NB, SW>(slot, Ws + t * kFusedW * SW, r, hb, acc);
      wave_lds_sync();  // the slot is read; the next relation may overwrite it
    }
    if (out == nullptr) continue;  // BWD without grad_hidden: only gy was wanted
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int64_t m = v0 + (reg & 3) + 8 * (reg >> 2) + 4 * hb;
      if (m >= num_rows) continue;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = nb * 32 + r;
        if (n >= out_w) continue;
        // forward epilogue (RelGraphConv, relgraphconv.py:186-190): + h_bias, then
        // + the self-loop message, in the reference's order
        float v = acc[nb][reg];
        if (bias) v += bias[n];
        if (addend) v += addend[m * out_w + n];
        __builtin_nontemporal_store(v, out + m * out_w + n);
      }
    }
  }
}

// The same fused layer-1 walk on 16-row tiles, 16 waves per CU (round 4).  The
// 32-row kernel above holds one 8-wave block per CU: W (80 KB at 4 + 1 matrices of
// 64 x 64) plus eight 8.3 KB slots fill the 160 KB LDS, so each SIMD has two waves to
// cover the gathers' latency with (0.52 of 8 TB/s past L2, 24 % MFMA busy, waves
// waiting 57 %).  Here a wave owns 16-row tiles and multiplies them by
// v_mfma_f32_16x16x4_f32 (same f32 rate): its slot is 4 KB, so sixteen slots and W fit
// one 1024-thread block -- four waves per SIMD, without re-walking the CSR.
//  * Slots and W are XOR-swizzled by float4 (no padding: 159744 B of LDS), so the MFMA
//    operand reads are conflict-free ds_read_b128: the k order inside the sum is
//    permuted (lane group kq covers k = 16 kq + 4 s + j over the 16 instructions of a
//    64-deep pass), which lets every lane take four k-steps of A and of B in one read.
//  * W is stored transposed, Wt[t][n][k], for the same reason.
//  * Two tiles per queue grab on the same eight queues (twice the tiles).
// Everything else -- equal edge shares per 16-lane group with in-order carries, the
// self-loop pass, gy stores, the epilogue -- is the 32-row kernel's.
constexpr int kR16Threads = 1024;
constexpr int kR16Grab = 4;

// float index of (row, col) in a 16 x 64 swizzled slot / a 64-float Wt row
__device__ __forceinline__ int swz(int row, int col) {
  return ((((col >> 2) ^ row) & 15) << 2) | (col & 3) | (col & ~63);
}

template <bool BWD, int NB16>
__global__ void __launch_bounds__(kR16Threads) k_rgcn_fused16(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ cols,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ eids, const float* __restrict__ w,
    const float* __restrict__ T, const float* __restrict__ W, int64_t ws_t, int64_t ws_k,
    int64_t ws_n, float* __restrict__ out, float* __restrict__ gy, int64_t num_rows, int R,
    int out_w, const float* __restrict__ bias, const float* __restrict__ addend,
    const float* __restrict__ Lw, unsigned* __restrict__ tile_ctr) {
  using f32x4 = __attribute__((ext_vector_type(4))) float;
  constexpr int SW = NB16 * 16;  // output columns held (out_w rounded up to 32)
  // row gathers in flight per lane: as many as fit 128 VGPRs without spills (the
  // backward keeps more state live; hipcc -Rpass-analysis=kernel-resource-usage)
  constexpr int GU = (!BWD && NB16 <= 4) ? 8 : ((BWD && NB16 == 8) ? 2 : 4);
  __shared__ float Ws[kFusedWsFloats];
  __shared__ float slots[16][16 * kFusedW];
  __shared__ float carries[16][3][kFusedW];
  const int RL = R + (Lw != nullptr);
  // Wt[t][n][k] (k swizzled by float4 against n & 15)
  for (int i = threadIdx.x; i < RL * kFusedW * SW; i += kR16Threads) {
    const int t = i / (kFusedW * SW), k = (i / SW) % kFusedW, n = i % SW;
    const float v = n >= out_w ? 0.0f
                               : (t < R ? W[t * ws_t + k * ws_k + n * ws_n] : Lw[k * ws_k + n * ws_n]);
    Ws[t * kFusedW * SW + n * kFusedW + swz(n & 15, k)] = v;
  }
  __syncthreads();  // the only block barrier
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = lane & 15, kq = lane >> 4;  // MFMA: A row / B, C column; k group
  const int g = lane >> 4, q = lane & 15;   // gather: 16-lane group, float4 column
  float* slot = slots[wv];
  float* carry = carries[wv][0];
  // the gathered table by a buffer resource: 32-bit byte offsets (the launcher takes this
  // kernel for tables under 4 GiB), one VGPR per gather in flight instead of two
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T), 0, -1, 0x00020000);
  const int64_t tiles = (num_rows + 15) / 16;
  const int nq = gridDim.x < 8 ? static_cast<int>(gridDim.x) : 8;
  const int64_t qid = blockIdx.x % nq;
  unsigned* ctr = tile_ctr + qid * kCtrStride;
  const int64_t qtiles = tiles > qid ? (tiles - qid + nq - 1) / nq : 0;
  for (int64_t k0 = 0;;) {
    if ((k0 & (kR16Grab - 1)) == 0) {
      unsigned tv = 0;
      if (lane == 0) tv = atomicAdd(ctr, static_cast<unsigned>(kR16Grab));
      k0 = static_cast<unsigned>(__builtin_amdgcn_readfirstlane(static_cast<int>(tv)));
    }
    if (k0 >= qtiles) break;
    const int64_t tile = qid + nq * k0;
    ++k0;
    const int64_t v0 = tile * 16;
    const int tile_rows = num_rows - v0 < 16 ? static_cast<int>(num_rows - v0) : 16;
    f32x4 acc[NB16];
#pragma unroll
    for (int nb = 0; nb < NB16; ++nb) acc[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int t = 0; t < RL; ++t) {
      if (t == R) {
        // self-loop: the tile's own rows of T (coalesced), 4 rows per group
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * g + i;
          const int64_t v = v0 + row;
          const float4 a = v < num_rows ? *reinterpret_cast<const float4*>(T + v * kFusedW + 4 * q)
                                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          *reinterpret_cast<float4*>(slot + row * kFusedW + swz(row, 4 * q)) = a;
        }
      } else {
        const int64_t base = static_cast<int64_t>(t) * num_rows + v0;
        const int64_t pb = ptr[base], pe = ptr[base + tile_rows];
        if (!BWD && pb == pe) continue;  // no relation-t edge into the tile
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * g + i;
          *reinterpret_cast<float4*>(slot + row * kFusedW + swz(row, 4 * q)) =
              make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        const int64_t share = (pe - pb + 3) / 4;
        const int64_t gb = pb + g * share < pe ? pb + g * share : pe;
        const int64_t ge = gb + share < pe ? gb + share : pe;
        const bool cont = gb < ge && gb > pb && rows[gb - 1] == rows[gb];  // never group 0
        bool first = true;
        int crow = -1;
        float4 a4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        int cur = -1;
        auto flush = [&]() {
          float* d = (first && cont) ? carry + (g - 1) * kFusedW + 4 * q
                                     : slot + cur * kFusedW + swz(cur, 4 * q);
          if (first && cont) crow = cur;
          *reinterpret_cast<float4*>(d) = a4;
          first = false;
        };
        for (int64_t p = gb; p < ge; p += 16) {
          const int n = ge - p < 16 ? static_cast<int>(ge - p) : 16;
          int my_col = 0, my_row = -1;
          float my_w = 0.0f;
          if (q < n) {
            my_col = cols[p + q];
            my_row = static_cast<int>(rows[p + q] - base);
            my_w = w[eids ? eids[p + q] : p + q];
          }
#pragma unroll
          for (int j0 = 0; j0 < 16; j0 += GU) {
            float4 x[GU];
            float wj[GU];
            int rj[GU];
#pragma unroll
            for (int u = 0; u < GU; ++u) {
              const int c = row_bcast16(my_col, j0 + u);
              rj[u] = row_bcast16(my_row, j0 + u);
              wj[u] = __int_as_float(row_bcast16(__float_as_int(my_w), j0 + u));
              const uint32_t off = (static_cast<uint32_t>(c) * kFusedW + 4u * q) * 4u;
              typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
              const u32x4v r4 = __builtin_amdgcn_raw_buffer_load_b128(trs, static_cast<int>(off), 0, 0);
              x[u] = make_float4(__uint_as_float(r4.x), __uint_as_float(r4.y), __uint_as_float(r4.z),
                                 __uint_as_float(r4.w));
            }
#pragma unroll
            for (int u = 0; u < GU; ++u) {
              if (rj[u] < 0) break;  // past the batch (group-uniform)
              if (rj[u] != cur) {
                if (cur >= 0) flush();
                a4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                cur = rj[u];
              }
              a4.x += wj[u] * x[u].x;
              a4.y += wj[u] * x[u].y;
              a4.z += wj[u] * x[u].z;
              a4.w += wj[u] * x[u].w;
            }
          }
        }
        if (cur >= 0) flush();
        wave_lds_sync();
        // carries into their rows, in group order (deterministic)
#pragma unroll
        for (int gg = 1; gg < 4; ++gg) {
          const int cr = __builtin_amdgcn_readlane(crow, gg * 16);
          if (cr >= 0) slot[cr * kFusedW + swz(cr, lane)] += carry[(gg - 1) * kFusedW + lane];
        }
      }
      wave_lds_sync();
      if constexpr (BWD) {
        // the slot's rows -> gy[v][t * 64 + c] (the weight gradients' operand)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * g + i;
          if (row >= tile_rows) break;
          const float4 v = *reinterpret_cast<const float4*>(slot + row * kFusedW + swz(row, 4 * q));
          float* d = gy + (v0 + row) * (static_cast<int64_t>(RL) * kFusedW) + t * kFusedW + 4 * q;
          __builtin_nontemporal_store(v.x, d);
          __builtin_nontemporal_store(v.y, d + 1);
          __builtin_nontemporal_store(v.z, d + 2);
          __builtin_nontemporal_store(v.w, d + 3);
        }
      }
      if (out != nullptr) {
        // acc[nb] += slot (16 x 64) . W_t (64 x 16 nb..): k = 16 kq + 4 s + j
        const float* wt = Ws + t * kFusedW * SW;
#pragma unroll 1
        for (int s4 = 0; s4 < 4; ++s4) {
          const int c = 16 * kq + 4 * s4;
          const float4 a = *reinterpret_cast<const float4*>(slot + m * kFusedW + swz(m, c));
#pragma unroll
          for (int nb = 0; nb < NB16; ++nb) {
            const int n = nb * 16 + m;
            const float4 b = *reinterpret_cast<const float4*>(wt + n * kFusedW + swz(m, c));
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[nb], 0, 0, 0);
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[nb], 0, 0, 0);
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[nb], 0, 0, 0);
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[nb], 0, 0, 0);
          }
        }
      }
      wave_lds_sync();  // the slot is read; the next relation may overwrite it
    }
    if (out == nullptr) continue;  // BWD without grad_hidden: only gy was wanted
    // C[row 4 kq + i][col nb * 16 + m]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t mrow = v0 + 4 * kq + i;
      if (mrow >= num_rows) continue;
#pragma unroll
      for (int nb = 0; nb < NB16; ++nb) {
        const int n = nb * 16 + m;
        if (n >= out_w) continue;
        float v = acc[nb][i];
        if (bias) v += bias[n];
        if (addend) v += addend[mrow * out_w + n];
        __builtin_nontemporal_store(v, out + mrow * out_w + n);
      }
    }
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

// out[i] += a[i]
__global__ void k_add_into(float* __restrict__ out, const float* __restrict__ a, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] += a[i];
}

unsigned grid1(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

// out[p] = v[idx[p]] (a per-edge operand permuted into a walk's position order),
// and out[p] = p
__global__ void k_gather_f32(const float* __restrict__ v, const int32_t* __restrict__ idx, int64_t n,
                             float* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < n; p += stride)
    out[p] = v[idx[p]];
}
__global__ void k_iota_i32(int32_t* __restrict__ out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < n; p += stride)
    out[p] = static_cast<int32_t>(p);
}

}  // namespace

void launch_gather_f32(const float* v, const int32_t* idx, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_f32, dim3(grid1(n)), dim3(kBlock), 0, s, v, idx, n, out);
}

void launch_iota_i32(int32_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_iota_i32, dim3(grid1(n)), dim3(kBlock), 0, s, out, n);
}

void launch_typed_ids(const int32_t* ids, const int32_t* eids, const int32_t* etypes, int64_t nnz,
                      int64_t mul, int mode, int32_t* out, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_typed_ids, dim3(grid1(nnz)), dim3(kBlock), 0, s, ids, eids, etypes, nnz, mul,
                     mode, out);
}

void launch_add_into(float* out, const float* a, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_add_into, dim3(grid1(n)), dim3(kBlock), 0, s, out, a, n);
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

namespace {

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <int NB, int KP>
void launch_rows(const float* A, int64_t lda, const float* B, int64_t b_rs, int64_t b_cs, float* C,
                 int64_t M, int64_t N, int64_t K, hipStream_t s) {
  const int64_t tiles = (M + 31) / 32;
  const int64_t want = (tiles + 7) / 8;
  const unsigned blocks = static_cast<unsigned>(want < 256 ? want : 256);  // one per CU
  hipLaunchKernelGGL((k_gemm_rows<NB, KP>), dim3(blocks), dim3(kGemmThreads), 0, s, A, lda, B, b_rs,
                     b_cs, C, M, static_cast<int>(N), static_cast<int>(K));
}

// k_gemm_rows when A is row-major with float4-loadable rows and B fits the LDS of one
// of the instances; false = not taken
bool try_rows(const float* A, int64_t a_rs, int64_t a_cs, const float* B, int64_t b_rs,
              int64_t b_cs, float* C, int64_t M, int64_t N, int64_t K, hipStream_t s) {
  if (a_cs != 1 || a_rs % 4 != 0 || K % 4 != 0 || !al16(A) || M < 4096) return false;
  if (N <= 256 && K <= 64) launch_rows<8, 64>(A, a_rs, B, b_rs, b_cs, C, M, N, K, s);
  else if (N <= 128 && K <= 128) launch_rows<4, 128>(A, a_rs, B, b_rs, b_cs, C, M, N, K, s);
  else if (N <= 64 && K <= 256) launch_rows<2, 256>(A, a_rs, B, b_rs, b_cs, C, M, N, K, s);
  else return false;
  return true;
}

template <int MB, int NB>
void launch_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t M,
               int64_t N, int64_t R, int64_t max_blocks, float* partials, hipStream_t s) {
  int64_t nb = max_blocks < 512 ? max_blocks : 512;
  int64_t rpb = ((R + nb - 1) / nb + kSlice - 1) / kSlice * kSlice;
  nb = (R + rpb - 1) / rpb;
  hipLaunchKernelGGL((k_gemm_tn<MB, NB>), dim3(static_cast<unsigned>(nb)), dim3(kGemmThreads), 0, s,
                     A, lda, B, ldb, partials, R, static_cast<int>(M), static_cast<int>(N), rpb);
  hipLaunchKernelGGL(k_sum_splits, dim3(grid1(M * N)), dim3(kBlock), 0, s, partials,
                     static_cast<int>(nb), M * N, C);
}

// k_gemm_tn for C = A^T B with A (K x M) and B (K x N) row-major (a_rs == 1, b_cs == 1),
// K the long dimension, through the caller's `splits` partial buffers
bool try_tn(const float* A, int64_t a_rs, int64_t a_cs, const float* B, int64_t b_rs,
            int64_t b_cs, float* C, int64_t M, int64_t N, int64_t K, int64_t splits,
            float* partials, hipStream_t s) {
  if (a_rs != 1 || b_cs != 1 || splits < 2 || partials == nullptr || K < 4096) return false;
  if (M % 4 != 0 || N % 4 != 0 || a_cs % 4 != 0 || b_rs % 4 != 0 || !al16(A) || !al16(B))
    return false;
  if (M <= 64 && N <= 256) launch_tn<2, 8>(A, a_cs, B, b_rs, C, M, N, K, splits, partials, s);
  else if (M <= 64 && N <= 320) launch_tn<2, 10>(A, a_cs, B, b_rs, C, M, N, K, splits, partials, s);
  else if (M <= 128 && N <= 128) launch_tn<4, 4>(A, a_cs, B, b_rs, C, M, N, K, splits, partials, s);
  else if (M <= 256 && N <= 64) launch_tn<8, 2>(A, a_cs, B, b_rs, C, M, N, K, splits, partials, s);
  else return false;
  return true;
}

}  // namespace

// Tile height of the fused layer-1 kernels: 16 (k_rgcn_fused16, 16 waves per CU) or,
// with DGLMI_RGCN_TILE=32, the 8-wave 32-row kernel (A/B and fallback).
int rgcn_tile_rows() {
  const char* e = std::getenv("DGLMI_RGCN_TILE");  // read per launch: tests switch it
  return e != nullptr && std::atoi(e) == 32 ? 32 : 16;
}

bool rgcn_fused_ok(int64_t gathered_w, int64_t out_w, int64_t R) {
  if (gathered_w != kFusedW || out_w < 1 || out_w > 128 || R < 1) return false;
  const int64_t nb = out_w <= 32 ? 1 : (out_w <= 64 ? 2 : 4);
  return R * kFusedW * nb * 32 <= kFusedWsFloats;
}

void launch_rgcn_fused(bool bwd, const int32_t* ptr, const int32_t* cols, const int32_t* rows,
                       const int32_t* eids, const float* w, const float* T, const float* W,
                       int64_t ws_t, int64_t ws_k, int64_t ws_n, float* out, float* gy,
                       int64_t num_rows, int64_t R, int64_t out_w, hipStream_t s,
                       const float* bias, const float* addend, const float* loop_w,
                       int64_t t_rows) {
  if (num_rows <= 0) return;
  if (t_rows < 0) t_rows = num_rows;
  const int64_t tiles = (num_rows + 31) / 32;
  const int64_t want = (tiles + 7) / 8;
  const dim3 grid(static_cast<unsigned>(want < 256 ? want : 256)), block(kGemmThreads);
  const int Ri = static_cast<int>(R), ow = static_cast<int>(out_w);
  // the tile queue's counter: stream-ordered, zeroed before and released after
  unsigned* ctr = nullptr;
  const size_t ctr_bytes = 8 * kCtrStride * sizeof(unsigned);
  if (hipMallocAsync(reinterpret_cast<void**>(&ctr), ctr_bytes, s) != hipSuccess ||
      hipMemsetAsync(ctr, 0, ctr_bytes, s) != hipSuccess)
    throw std::runtime_error("rgcn fused: tile counter allocation failed");
  // gathered table T: the rows of the relation-major walk's columns (num_rows of them
  // forward, the source rows backward: at most the larger of the two row counts)
  if (rgcn_tile_rows() == 16 && (num_rows + 1) * kFusedW * 4 < (int64_t(1) << 32) &&
      t_rows * kFusedW * 4 < (int64_t(1) << 32)) {
    const int64_t t16 = (num_rows + 15) / 16;
    const int64_t want16 = (t16 + 15) / 16;
    const dim3 grid16(static_cast<unsigned>(want16 < 256 ? want16 : 256)), block16(kR16Threads);
#define DGLMI_RGCN_FUSED16(B_, NB_)                                                               \
  hipLaunchKernelGGL((k_rgcn_fused16<B_, NB_>), grid16, block16, 0, s, ptr, cols, rows, eids, w, T, \
                     W, ws_t, ws_k, ws_n, out, gy, num_rows, Ri, ow, bias, addend, loop_w, ctr)
    if (bwd) {
      if (out_w <= 32) DGLMI_RGCN_FUSED16(true, 2);
      else if (out_w <= 64) DGLMI_RGCN_FUSED16(true, 4);
      else DGLMI_RGCN_FUSED16(true, 8);
    } else {
      if (out_w <= 32) DGLMI_RGCN_FUSED16(false, 2);
      else if (out_w <= 64) DGLMI_RGCN_FUSED16(false, 4);
      else DGLMI_RGCN_FUSED16(false, 8);
    }
#undef DGLMI_RGCN_FUSED16
    (void)hipFreeAsync(ctr, s);
    return;
  }
#define DGLMI_RGCN_FUSED(B_, NB_)                                                               \
  hipLaunchKernelGGL((k_rgcn_fused<B_, NB_>), grid, block, 0, s, ptr, cols, rows, eids, w, T, W, \
                     ws_t, ws_k, ws_n, out, gy, num_rows, Ri, ow, bias, addend, loop_w, ctr)
  if (bwd) {
    if (out_w <= 32) DGLMI_RGCN_FUSED(true, 1);
    else if (out_w <= 64) DGLMI_RGCN_FUSED(true, 2);
    else DGLMI_RGCN_FUSED(true, 4);
  } else {
    if (out_w <= 32) DGLMI_RGCN_FUSED(false, 1);
    else if (out_w <= 64) DGLMI_RGCN_FUSED(false, 2);
    else DGLMI_RGCN_FUSED(false, 4);
  }
#undef DGLMI_RGCN_FUSED
  (void)hipFreeAsync(ctr, s);
}

void launch_gemm(const float* A, int64_t a_rs, int64_t a_cs, const float* B, int64_t b_rs,
                 int64_t b_cs, float* C, int64_t M, int64_t N, int64_t K, int64_t splits,
                 float* partials, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  if (K <= 0) {
    launch_fill(C, M * N, 0.0f, s);
    return;
  }
  if (try_rows(A, a_rs, a_cs, B, b_rs, b_cs, C, M, N, K, s)) return;
  if (try_tn(A, a_rs, a_cs, B, b_rs, b_cs, C, M, N, K, splits, partials, s)) return;
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
