// Graph ingestion: COO -> CSR, CSR transpose, CSR row expansion.
//
// Host versions restate aten::COOToCSR (array/cpu/spmat_op_impl_coo.cc:230-283)
// and aten::CSRTranspose (array/cpu/spmat_op_impl.cc:323-369): stable counting
// sorts, so the resulting arrays are bit-identical to the reference's.
// The device version builds the same arrays on the GPU with a stable LSD
// radix sort of (row, position) pairs -- stability gives the identical
// within-row order -- so a multi-hundred-million-edge graph never needs a
// CPU CSR build and a host-to-device copy (the reference builds on the CPU
// and copies, immutable_graph.cc:548-559).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "internal.h"

namespace {

template <typename I>
void coo_to_csr(int64_t n, int64_t nnz, const I* row, const I* col, const I* data, I* bp, I* bi,
                I* bx) {
  std::fill(bp, bp + n, I(0));
  for (int64_t i = 0; i < nnz; ++i) bp[row[i]]++;
  I cum = 0;
  for (int64_t i = 0; i < n; ++i) {
    const I t = bp[i];
    bp[i] = cum;
    cum += t;
  }
  bp[n] = static_cast<I>(nnz);
  for (int64_t i = 0; i < nnz; ++i) {
    const I r = row[i];
    bi[bp[r]] = col[i];
    bx[bp[r]] = data ? data[i] : static_cast<I>(i);
    bp[r]++;
  }
  I last = 0;
  for (int64_t i = 0; i <= n; ++i) {
    const I t = bp[i];
    bp[i] = last;
    last = t;
  }
}

template <typename I>
void csr_transpose(int64_t n, int64_t m, const I* ap, const I* aj, const I* ax, I* bp, I* bi,
                   I* bx) {
  const int64_t nnz = ap[n];
  std::fill(bp, bp + m, I(0));
  for (int64_t j = 0; j < nnz; ++j) bp[aj[j]]++;
  I cum = 0;
  for (int64_t i = 0; i < m; ++i) {
    const I t = bp[i];
    bp[i] = cum;
    cum += t;
  }
  bp[m] = static_cast<I>(nnz);
  for (int64_t i = 0; i < n; ++i) {
    for (I j = ap[i]; j < ap[i + 1]; ++j) {
      const I d = aj[j];
      bi[bp[d]] = static_cast<I>(i);
      bx[bp[d]] = ax ? ax[j] : j;
      bp[d]++;
    }
  }
  I last = 0;
  for (int64_t i = 0; i <= m; ++i) {
    const I t = bp[i];
    bp[i] = last;
    last = t;
  }
}

__global__ void k_iota(int32_t* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = static_cast<int32_t>(i);
}

__global__ void k_gather_cols(const int32_t* __restrict__ perm, const int32_t* __restrict__ col,
                              const int32_t* __restrict__ data, int32_t* __restrict__ indices,
                              int32_t* __restrict__ out_data, int64_t nnz) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
    const int32_t p = perm[i];
    indices[i] = col[p];
    out_data[i] = data ? data[p] : p;
  }
}

// indptr from the sorted row keys: position i opens every row in (key[i-1], key[i]].
__global__ void k_indptr_from_sorted(const int32_t* __restrict__ key, int64_t nnz, int64_t n,
                                     int32_t* __restrict__ indptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= nnz; i += stride) {
    const int64_t lo = i == 0 ? 0 : (int64_t)key[i - 1] + 1;
    const int64_t hi = i == nnz ? n : (int64_t)key[i];
    for (int64_t r = lo; r <= hi; ++r) indptr[r] = static_cast<int32_t>(i);
  }
}

__global__ void k_mark_row_starts(const int32_t* __restrict__ indptr, int64_t n,
                                  int32_t* __restrict__ rows) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride)
    if (indptr[r + 1] > indptr[r]) rows[indptr[r]] = static_cast<int32_t>(r);
}

struct MaxOp {
  __device__ __forceinline__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; }
};

unsigned grid_of(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return static_cast<unsigned>(b);
}

int bits_for(int64_t n) {
  int b = 1;
  while ((int64_t(1) << b) < n && b < 31) ++b;
  return b;
}

size_t sort_temp_bytes(int64_t n, int64_t nnz) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const int32_t*>(nullptr),
                                     static_cast<int32_t*>(nullptr),
                                     static_cast<const int32_t*>(nullptr),
                                     static_cast<int32_t*>(nullptr), static_cast<int>(nnz), 0,
                                     bits_for(n));
  return bytes;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ---- 64-bit graphs (2^31 or more edges): int64 offsets and edge ids ----------
// COO -> CSR as a stable counting sort by row done in batches of at most 2^30
// positions, in position order.  Row counts (atomics) and their exclusive scan give
// indptr; each batch is sorted by (row, position) with the same stable radix sort
// as the int32 path (int item counts), and its run of row r is written after the
// runs of the earlier batches (a per-row fill cursor), so every row keeps its
// positions ascending: bit-identical to COOToCSR with int64 arrays.
constexpr int64_t kBatch64 = int64_t(1) << 30;

__global__ void k_count_rows64(const int32_t* __restrict__ row, int64_t nnz,
                               unsigned long long* __restrict__ cnt) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride)
    atomicAdd(cnt + row[i], 1ull);
}

// rs[i] = i where a run of equal keys starts, else 0 (a max-scan then gives every
// position its run's start)
__global__ void k_run_starts(const int32_t* __restrict__ key, int64_t n, int32_t* __restrict__ rs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    rs[i] = (i == 0 || key[i] != key[i - 1]) ? static_cast<int32_t>(i) : 0;
}

__global__ void k_scatter_batch64(const int32_t* __restrict__ key, const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ rs, int64_t n, int64_t start,
                                  const int32_t* __restrict__ col, const int64_t* __restrict__ data,
                                  const int64_t* __restrict__ fill, int32_t* __restrict__ indices,
                                  int64_t* __restrict__ out_data) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t p = start + perm[i];
    const int64_t dest = fill[key[i]] + (i - rs[i]);
    indices[dest] = col[p];
    out_data[dest] = data ? data[p] : p;
  }
}

// the last position of each run advances its row's cursor by the run's length
__global__ void k_advance_fill(const int32_t* __restrict__ key, const int32_t* __restrict__ rs,
                               int64_t n, int64_t* __restrict__ fill) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    if (i == n - 1 || key[i + 1] != key[i]) fill[key[i]] += i - rs[i] + 1;
}

__global__ void k_mark_row_starts64(const int64_t* __restrict__ indptr, int64_t n,
                                    int32_t* __restrict__ rows) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride)
    if (indptr[r + 1] > indptr[r]) rows[indptr[r]] = static_cast<int32_t>(r);
}

// carry of a batched max-scan: the batch's first element takes the previous
// batch's final value into account
__global__ void k_scan_carry(int32_t* __restrict__ v, int64_t start) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && v[start - 1] > v[start]) v[start] = v[start - 1];
}

struct Ws64 {
  size_t fill, keys, perm_in, perm_out, rs, temp, total;
};

Ws64 ws64_layout(int64_t n, int64_t nnz) {
  const int64_t b = nnz < kBatch64 ? nnz : kBatch64;
  size_t sort_b = 0, scan_b = 0, max_b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, static_cast<const int32_t*>(nullptr),
                                           static_cast<int32_t*>(nullptr),
                                           static_cast<const int32_t*>(nullptr),
                                           static_cast<int32_t*>(nullptr), static_cast<int>(b), 0,
                                           bits_for(n));
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, static_cast<const int64_t*>(nullptr),
                                         static_cast<int64_t*>(nullptr), static_cast<int>(n + 1));
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, max_b, static_cast<int32_t*>(nullptr),
                                          static_cast<int32_t*>(nullptr), MaxOp(), static_cast<int>(b));
  Ws64 w;
  w.fill = 0;
  w.keys = w.fill + align256((n + 1) * sizeof(int64_t));
  w.perm_in = w.keys + align256(b * sizeof(int32_t));
  w.perm_out = w.perm_in + align256(b * sizeof(int32_t));
  w.rs = w.perm_out + align256(b * sizeof(int32_t));
  w.temp = w.rs + align256(b * sizeof(int32_t));
  w.total = w.temp + align256(std::max(sort_b, std::max(scan_b, max_b)));
  return w;
}

thread_local std::string g_ingest_error;

// rows of R = 4 << SH floats: 1 << SH lanes per row, one float4 each, so one load
// instruction reads 64 / (1 << SH) whole rows (one cache-line request per row, not one
// per float4); two float4 in flight per lane
template <int SH>
__global__ void __launch_bounds__(256) k_gather_rows_v4(const float4* __restrict__ src,
                                                        const int32_t* __restrict__ i32,
                                                        const int64_t* __restrict__ i64,
                                                        int64_t n, float4* __restrict__ out) {
  const int64_t total = n << SH;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += 2 * stride) {
    const int64_t q2 = q + stride;
    const int64_t i = q >> SH, i2 = q2 >> SH;
    const int64_t j = i32 != nullptr ? static_cast<int64_t>(i32[i]) : i64[i];
    const int64_t c = q & ((1 << SH) - 1);
    const float4 v = src[(j << SH) + c];
    float4 v2;
    if (q2 < total) {
      const int64_t j2 = i32 != nullptr ? static_cast<int64_t>(i32[i2]) : i64[i2];
      v2 = src[(j2 << SH) + (q2 & ((1 << SH) - 1))];
    }
    out[q] = v;
    if (q2 < total) out[q2] = v2;
  }
}

// any other row width: one lane per row
__global__ void __launch_bounds__(256) k_gather_rows(const float* __restrict__ src, int64_t R,
                                                     const int32_t* __restrict__ i32,
                                                     const int64_t* __restrict__ i64, int64_t n,
                                                     float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t j = i32 != nullptr ? static_cast<int64_t>(i32[i]) : i64[i];
    const float* s = src + j * R;
    float* o = out + i * R;
    for (int64_t c = 0; c < R; ++c) o[c] = s[c];
  }
}

}  // namespace

extern "C" {

int DGLMICOOToCSR(int64_t num_rows, int64_t nnz, const int64_t* row, const int64_t* col,
                  const int64_t* data, int64_t* indptr, int64_t* indices, int64_t* out_data) {
  if (num_rows < 0 || nnz < 0 || indptr == nullptr) return -1;
  for (int64_t i = 0; i < nnz; ++i)
    if (row[i] < 0 || row[i] >= num_rows) return -1;
  coo_to_csr<int64_t>(num_rows, nnz, row, col, data, indptr, indices, out_data);
  return 0;
}

int DGLMICSRTranspose(int64_t num_rows, int64_t num_cols, const int64_t* indptr,
                      const int64_t* indices, const int64_t* data, int64_t* t_indptr,
                      int64_t* t_indices, int64_t* t_data) {
  if (num_rows < 0 || num_cols < 0 || indptr == nullptr || t_indptr == nullptr) return -1;
  for (int64_t j = 0; j < indptr[num_rows]; ++j)
    if (indices[j] < 0 || indices[j] >= num_cols) return -1;
  csr_transpose<int64_t>(num_rows, num_cols, indptr, indices, data, t_indptr, t_indices, t_data);
  return 0;
}

int64_t DGLMICOOToCSRDeviceWorkspaceBytes(int64_t num_rows, int64_t nnz) {
  if (nnz <= 0) return 256;
  return static_cast<int64_t>(3 * align256(nnz * sizeof(int32_t)) +
                              align256(sort_temp_bytes(num_rows, nnz)));
}

int DGLMICOOToCSRDevice(int64_t num_rows, int64_t nnz, const int32_t* row, const int32_t* col,
                        const int32_t* data, int32_t* indptr, int32_t* indices, int32_t* out_data,
                        void* workspace, int64_t workspace_bytes, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (num_rows < 0 || nnz < 0 || nnz > INT32_MAX || num_rows >= INT32_MAX) return -1;
  if (nnz == 0) {
    dglmi::launch_fill_i32(indptr, num_rows + 1, 0, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (workspace_bytes < DGLMICOOToCSRDeviceWorkspaceBytes(num_rows, nnz)) return -1;
  char* ws = static_cast<char*>(workspace);
  const size_t seg = align256(nnz * sizeof(int32_t));
  int32_t* keys_out = reinterpret_cast<int32_t*>(ws);
  int32_t* perm_in = reinterpret_cast<int32_t*>(ws + seg);
  int32_t* perm_out = reinterpret_cast<int32_t*>(ws + 2 * seg);
  void* temp = ws + 3 * seg;
  size_t temp_bytes = sort_temp_bytes(num_rows, nnz);
  hipLaunchKernelGGL(k_iota, dim3(grid_of(nnz)), dim3(256), 0, s, perm_in, nnz);
  if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, row, keys_out, perm_in, perm_out,
                                         static_cast<int>(nnz), 0, bits_for(num_rows), s) !=
      hipSuccess)
    return -1;
  hipLaunchKernelGGL(k_gather_cols, dim3(grid_of(nnz)), dim3(256), 0, s, perm_out, col, data,
                     indices, out_data, nnz);
  hipLaunchKernelGGL(k_indptr_from_sorted, dim3(grid_of(nnz + 1)), dim3(256), 0, s, keys_out, nnz,
                     num_rows, indptr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int64_t DGLMICOOToCSRDevice64WorkspaceBytes(int64_t num_rows, int64_t nnz) {
  if (nnz <= 0 || num_rows < 0) return 256;
  return static_cast<int64_t>(ws64_layout(num_rows, nnz).total);
}

int DGLMICOOToCSRDevice64(int64_t num_rows, int64_t nnz, const int32_t* row, const int32_t* col,
                          const int64_t* data, int64_t* indptr, int32_t* indices, int64_t* out_data,
                          void* workspace, int64_t workspace_bytes, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (num_rows < 0 || nnz < 0 || num_rows >= INT32_MAX || indptr == nullptr) return -1;
  if (nnz == 0) {
    if (hipMemsetAsync(indptr, 0, (num_rows + 1) * sizeof(int64_t), s) != hipSuccess) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const Ws64 w = ws64_layout(num_rows, nnz);
  if (workspace == nullptr || workspace_bytes < static_cast<int64_t>(w.total)) return -1;
  char* ws = static_cast<char*>(workspace);
  int64_t* fill = reinterpret_cast<int64_t*>(ws + w.fill);
  int32_t* keys = reinterpret_cast<int32_t*>(ws + w.keys);
  int32_t* perm_in = reinterpret_cast<int32_t*>(ws + w.perm_in);
  int32_t* perm_out = reinterpret_cast<int32_t*>(ws + w.perm_out);
  int32_t* rs = reinterpret_cast<int32_t*>(ws + w.rs);
  void* temp = ws + w.temp;
  const size_t temp_cap = w.total - w.temp;
  // row counts -> indptr (exclusive scan over num_rows + 1 entries, the last zero)
  if (hipMemsetAsync(fill, 0, (num_rows + 1) * sizeof(int64_t), s) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_count_rows64, dim3(grid_of(nnz)), dim3(256), 0, s, row, nnz,
                     reinterpret_cast<unsigned long long*>(fill));
  size_t tb = temp_cap;
  if (hipcub::DeviceScan::ExclusiveSum(temp, tb, fill, indptr, static_cast<int>(num_rows + 1), s) !=
      hipSuccess)
    return -1;
  if (hipMemcpyAsync(fill, indptr, num_rows * sizeof(int64_t), hipMemcpyDeviceToDevice, s) !=
      hipSuccess)
    return -1;
  for (int64_t start = 0; start < nnz; start += kBatch64) {
    const int64_t nb = std::min(kBatch64, nnz - start);
    hipLaunchKernelGGL(k_iota, dim3(grid_of(nb)), dim3(256), 0, s, perm_in, nb);
    tb = temp_cap;
    if (hipcub::DeviceRadixSort::SortPairs(temp, tb, row + start, keys, perm_in, perm_out,
                                           static_cast<int>(nb), 0, bits_for(num_rows), s) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_run_starts, dim3(grid_of(nb)), dim3(256), 0, s, keys, nb, rs);
    tb = temp_cap;
    if (hipcub::DeviceScan::InclusiveScan(temp, tb, rs, rs, MaxOp(), static_cast<int>(nb), s) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_scatter_batch64, dim3(grid_of(nb)), dim3(256), 0, s, keys, perm_out, rs, nb,
                       start, col, data, fill, indices, out_data);
    hipLaunchKernelGGL(k_advance_fill, dim3(grid_of(nb)), dim3(256), 0, s, keys, rs, nb, fill);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int DGLMICSRExpandRows64(const int64_t* indptr, int64_t num_rows, int64_t nnz, int32_t* rows,
                         void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nnz == 0) return 0;
  if (num_rows >= INT32_MAX) return -1;
  dglmi::launch_fill_i32(rows, nnz, 0, s);
  hipLaunchKernelGGL(k_mark_row_starts64, dim3(grid_of(num_rows)), dim3(256), 0, s, indptr, num_rows,
                     rows);
  const int64_t b = std::min(kBatch64, nnz);
  size_t temp_bytes = 0;
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, temp_bytes, rows, rows, MaxOp(), static_cast<int>(b),
                                          s);
  void* temp = nullptr;
  if (hipMallocAsync(&temp, temp_bytes, s) != hipSuccess) return -1;
  hipError_t e = hipSuccess;
  for (int64_t start = 0; start < nnz && e == hipSuccess; start += kBatch64) {
    const int64_t nb = std::min(kBatch64, nnz - start);
    if (start > 0) hipLaunchKernelGGL(k_scan_carry, dim3(1), dim3(64), 0, s, rows, start);
    size_t tb = temp_bytes;
    e = hipcub::DeviceScan::InclusiveScan(temp, tb, rows + start, rows + start, MaxOp(),
                                          static_cast<int>(nb), s);
  }
  (void)hipFreeAsync(temp, s);
  if (e != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int DGLMICSRExpandRows(const int32_t* indptr, int64_t num_rows, int64_t nnz, int32_t* rows,
                       void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nnz == 0) return 0;
  dglmi::launch_fill_i32(rows, nnz, 0, s);
  hipLaunchKernelGGL(k_mark_row_starts, dim3(grid_of(num_rows)), dim3(256), 0, s, indptr, num_rows,
                     rows);
  size_t temp_bytes = 0;
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, temp_bytes, rows, rows, MaxOp(), static_cast<int>(nnz),
                                    s);
  void* temp = nullptr;
  if (hipMallocAsync(&temp, temp_bytes, s) != hipSuccess) return -1;
  const hipError_t e = hipcub::DeviceScan::InclusiveScan(temp, temp_bytes, rows, rows, MaxOp(),
                                                         static_cast<int>(nnz), s);
  (void)hipFreeAsync(temp, s);
  if (e != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// out[i, :] = src[index[i], :], rows of R floats: a per-edge operand put into a walk's
// position order.  Rows of 4, 8, .. 256 floats: float4 slices, a row's slices on
// adjacent lanes (k_gather_rows_v4); other widths one lane per row.  torch's
// index_select on a (114.6 M, 8, 1) tensor took 12 ms.
int DGLMIGatherRows(const float* src, int64_t row_floats, const void* index, int index_bits,
                    int64_t n, float* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n == 0 || row_floats == 0) return 0;
  if (src == nullptr || index == nullptr || out == nullptr || row_floats < 0 || n < 0 ||
      (index_bits != 32 && index_bits != 64))
    return -1;
  const int32_t* i32 = index_bits == 32 ? static_cast<const int32_t*>(index) : nullptr;
  const int64_t* i64 = index_bits == 64 ? static_cast<const int64_t*>(index) : nullptr;
  int sh = -1;  // row_floats = 4 << sh, sh <= 6
  for (int k = 0; k <= 6; ++k)
    if (row_floats == (int64_t{4} << k)) sh = k;
  const bool v4 = sh >= 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  auto grid_of_items = [](int64_t items) {
    return dim3(static_cast<unsigned>(std::min<int64_t>((items + 255) / 256, 65536)));
  };
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* o4 = reinterpret_cast<float4*>(out);
  const dim3 g4 = grid_of_items(((n << (sh < 0 ? 0 : sh)) + 1) / 2), blk(256);
  if (!v4) {
    hipLaunchKernelGGL(k_gather_rows, grid_of_items(n), blk, 0, s, src, row_floats, i32, i64, n, out);
  } else {
    switch (sh) {
      case 0: hipLaunchKernelGGL(k_gather_rows_v4<0>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      case 1: hipLaunchKernelGGL(k_gather_rows_v4<1>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      case 2: hipLaunchKernelGGL(k_gather_rows_v4<2>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      case 3: hipLaunchKernelGGL(k_gather_rows_v4<3>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      case 4: hipLaunchKernelGGL(k_gather_rows_v4<4>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      case 5: hipLaunchKernelGGL(k_gather_rows_v4<5>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
      default: hipLaunchKernelGGL(k_gather_rows_v4<6>, g4, blk, 0, s, s4, i32, i64, n, o4); break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Partitioning (no METIS here): Linear Deterministic Greedy, streaming over
// nodes in id order on the symmetrised adjacency.  Node v goes to the part
// maximising |N(v) ∩ P| * (1 - |P| / C), C = ceil(n / k) * (1 + slack); ties
// and neighbourless nodes go to the least-loaded part.  Deterministic.
// ---------------------------------------------------------------------------
extern "C" int DGLMIPartitionLDG(int64_t num_nodes, const int64_t* indptr, const int64_t* indices,
                                 int32_t num_parts, double slack, int64_t* assign) {
  if (num_nodes < 0 || num_parts < 1 || indptr == nullptr || assign == nullptr) return -1;
  std::vector<int64_t> size(num_parts, 0);
  std::vector<int64_t> cnt(num_parts, 0);
  const double cap = std::ceil(static_cast<double>(num_nodes) / num_parts) * (1.0 + slack);
  for (int64_t v = 0; v < num_nodes; ++v) assign[v] = -1;
  for (int64_t v = 0; v < num_nodes; ++v) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int64_t j = indptr[v]; j < indptr[v + 1]; ++j) {
      const int64_t u = indices[j];
      if (u >= 0 && u < num_nodes && assign[u] >= 0) cnt[assign[u]]++;
    }
    int best = -1;
    double best_score = -1.0;
    for (int p = 0; p < num_parts; ++p) {
      if (size[p] >= cap) continue;
      const double score = cnt[p] * (1.0 - size[p] / cap);
      if (best < 0 || score > best_score || (score == best_score && size[p] < size[best])) {
        best = p;
        best_score = score;
      }
    }
    if (best < 0) best = static_cast<int>(std::min_element(size.begin(), size.end()) - size.begin());
    assign[v] = best;
    size[best]++;
  }
  return 0;
}
