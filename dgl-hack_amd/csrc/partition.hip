// Graph partitioning on the device: balanced label propagation (no METIS here).
//
// The reference partitions with METIS k-way on the symmetrised graph
// (src/graph/metis_partition.cc:19-66, called by python/dgl/transform.py:
// 589-630 after to_bidirected).  METIS is a host library the image lacks, and a
// host pass over a 200 M-edge graph would be the slowest step of a multi-GPU
// run, so the partitioner runs where the graph already is: in HBM, on the in-
// and out-CSR every graph carries (their union IS the symmetrised adjacency, no
// extra copy).  One round, synchronous and deterministic:
//
//   score  every node counts its neighbours' parts (a 16-lane group per node,
//          histogram in LDS with integer atomics; nodes of degree >= kHeavy get
//          a whole workgroup) and proposes the most frequent part when it beats
//          its own strictly (ties: the lighter part, then the lower id).  Only
//          the nodes of one hash half propose per round, so two neighbours do
//          not swap back and forth;
//   admit  proposals into part p are admitted in the order of a counter-based
//          hash of (node, round, seed) until the part's room
//          (1 + slack) * total_weight / k - load[p] is used up -- exactly, with
//          two passes of 256-bin weight histograms per part over the hash
//          (the candidates of the bin that straddles the room in the finer
//          pass are all turned away), so a part never exceeds its cap and the
//          result does not depend on the order atomics land in;
//   apply  admitted nodes take their new part.
//
// Part loads are integer sums (atomics on int64), so they are exact and
// order-independent.  Statistics (cut edges, loads) come from one more pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kGroup = 16;                     // lanes per light node
constexpr int kGroupsPerBlock = kBlock / kGroup;
constexpr int kMaxParts = 64;
constexpr int64_t kHeavy = 4096;               // symmetric degree of a "heavy" node

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// 32-bit admission priority of (node, round)
__device__ __forceinline__ uint32_t admit_hash(int64_t v, int round, uint64_t seed) {
  const uint64_t h = splitmix(splitmix(seed ^ (uint64_t(1) << 56)) ^
                              (static_cast<uint64_t>(round) << 40) ^ static_cast<uint64_t>(v));
  return static_cast<uint32_t>(h >> 32);
}

// signed 64-bit add through the unsigned atomic (two's complement wraps exactly)
__device__ __forceinline__ void add_ll(long long* p, long long v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(v));
}

struct LpArgs {
  const int32_t* in_ptr;
  const int32_t* in_idx;
  const int32_t* out_ptr;
  const int32_t* out_idx;
  int64_t n;
  int k;
  const int32_t* label;
  const int32_t* weight;            // NULL = 1 per node
  const long long* load;            // k
  int round;
  uint64_t seed;
  int32_t* want;                    // n: proposed part or -1
  unsigned long long* hist_a;       // k x 256: proposed weight per (part, top hash byte)
};

__device__ __forceinline__ int64_t sym_degree(const LpArgs& a, int64_t v) {
  return (int64_t)(a.in_ptr[v + 1] - a.in_ptr[v]) + (a.out_ptr[v + 1] - a.out_ptr[v]);
}

// count the parts of v's neighbours (self-loops ignored) into hist, lanes [lane, .., step)
__device__ __forceinline__ void count_parts(const LpArgs& a, int64_t v, int lane, int step,
                                            int* hist) {
  for (int dir = 0; dir < 2; ++dir) {
    const int32_t* ptr = dir == 0 ? a.in_ptr : a.out_ptr;
    const int32_t* idx = dir == 0 ? a.in_idx : a.out_idx;
    const int64_t beg = ptr[v], end = ptr[v + 1];
    int64_t j = beg + lane;
    // four neighbours in flight per lane
    for (; j + 3 * step < end; j += 4 * step) {
      const int32_t u0 = idx[j], u1 = idx[j + step], u2 = idx[j + 2 * step], u3 = idx[j + 3 * step];
      const int32_t l0 = a.label[u0], l1 = a.label[u1], l2 = a.label[u2], l3 = a.label[u3];
      if (u0 != v) atomicAdd(&hist[l0], 1);
      if (u1 != v) atomicAdd(&hist[l1], 1);
      if (u2 != v) atomicAdd(&hist[l2], 1);
      if (u3 != v) atomicAdd(&hist[l3], 1);
    }
    for (; j < end; j += step) {
      const int32_t u = idx[j];
      if (u != v) atomicAdd(&hist[a.label[u]], 1);
    }
  }
}

// one thread decides for v from the finished histogram
__device__ __forceinline__ void propose(const LpArgs& a, int64_t v, const int* hist) {
  const int cur = a.label[v];
  int best = cur;
  for (int p = 0; p < a.k; ++p) {
    if (p == best) continue;
    const int c = hist[p], cb = hist[best];
    if (c > cb || (c == cb && best != cur && (a.load[p] < a.load[best] ||
                                             (a.load[p] == a.load[best] && p < best))))
      best = p;
  }
  // move only on a strict gain, and only the nodes of this round's hash half
  const bool half = (splitmix(a.seed ^ static_cast<uint64_t>(v) ^
                              (static_cast<uint64_t>(a.round) << 48)) & 1) == 0;
  if (best != cur && hist[best] > hist[cur] && half) {
    a.want[v] = best;
    const uint32_t h = admit_hash(v, a.round, a.seed);
    atomicAdd(&a.hist_a[best * 256 + (h >> 24)],
              static_cast<unsigned long long>(a.weight ? a.weight[v] : 1));
  } else {
    a.want[v] = -1;
  }
}

__global__ void __launch_bounds__(kBlock) k_lp_score_light(LpArgs a) {
  __shared__ int hist[kGroupsPerBlock][kMaxParts];
  const int g = threadIdx.x / kGroup, lane = threadIdx.x % kGroup;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kGroupsPerBlock;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kGroupsPerBlock; base < a.n;
       base += stride) {
    const int64_t v = base + g;
    for (int p = lane; p < a.k; p += kGroup) hist[g][p] = 0;
    __syncthreads();
    const bool light = v < a.n && sym_degree(a, v) < kHeavy;
    if (light) count_parts(a, v, lane, kGroup, hist[g]);
    __syncthreads();
    if (light && lane == 0) propose(a, v, hist[g]);
    __syncthreads();
  }
}

// one workgroup per heavy node (list built on the host side of the call)
__global__ void __launch_bounds__(kBlock) k_lp_score_heavy(LpArgs a, const int32_t* heavy,
                                                           int64_t num_heavy) {
  __shared__ int hist[kMaxParts];
  for (int64_t i = blockIdx.x; i < num_heavy; i += gridDim.x) {
    const int64_t v = heavy[i];
    for (int p = threadIdx.x; p < a.k; p += kBlock) hist[p] = 0;
    __syncthreads();
    count_parts(a, v, threadIdx.x, kBlock, hist);
    __syncthreads();
    if (threadIdx.x == 0) propose(a, v, hist);
    __syncthreads();
  }
}

// cutoff of one histogram level per part (one thread per part): bins below cut[p]
// are admitted whole; rem[p] is the room left for bin cut[p] (refined by the next
// level, or turned away after the last)
__global__ void k_admit_cut(int k, const unsigned long long* hist, const long long* room_in,
                            const int32_t* parent_cut, int32_t* cut, long long* rem,
                            const long long* load, long long cap) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= k) return;
  long long room = room_in ? room_in[p] : cap - load[p];
  if (parent_cut && parent_cut[p] >= 256) {  // everything admitted a level up
    cut[p] = 256;
    rem[p] = room;
    return;
  }
  int b = 0;
  for (; b < 256; ++b) {
    const long long w = static_cast<long long>(hist[p * 256 + b]);
    if (w > room) break;
    room -= w;
  }
  cut[p] = b;
  rem[p] = room;
}

// second level: weights of the candidates in the straddling top-level bin, by the
// next hash byte
__global__ void __launch_bounds__(kBlock) k_admit_hist_b(int64_t n, const int32_t* want,
                                                         const int32_t* weight, int round,
                                                         uint64_t seed, const int32_t* cut_a,
                                                         unsigned long long* hist_b) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < n; v += stride) {
    const int p = want[v];
    if (p < 0) continue;
    const uint32_t h = admit_hash(v, round, seed);
    if (static_cast<int>(h >> 24) != cut_a[p]) continue;
    atomicAdd(&hist_b[p * 256 + ((h >> 16) & 255)],
              static_cast<unsigned long long>(weight ? weight[v] : 1));
  }
}

__global__ void __launch_bounds__(kBlock) k_lp_apply(int64_t n, int k, const int32_t* want,
                                                     int32_t* label, const int32_t* weight,
                                                     const int32_t* cut_a, const int32_t* cut_b,
                                                     int round, uint64_t seed, long long* delta) {
  __shared__ long long d[kMaxParts];
  for (int p = threadIdx.x; p < k; p += kBlock) d[p] = 0;
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < n; v += stride) {
    const int p = want[v];
    if (p < 0) continue;
    const uint32_t h = admit_hash(v, round, seed);
    const int ba = static_cast<int>(h >> 24), bb = static_cast<int>((h >> 16) & 255);
    if (!(ba < cut_a[p] || (ba == cut_a[p] && bb < cut_b[p]))) continue;
    const long long w = weight ? weight[v] : 1;
    add_ll(&d[label[v]], -w);
    add_ll(&d[p], w);
    label[v] = p;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < k; p += kBlock)
    if (d[p] != 0) add_ll(&delta[p], d[p]);
}

__global__ void __launch_bounds__(kBlock) k_part_loads(int64_t n, int k, const int32_t* label,
                                                       const int32_t* weight, long long* load,
                                                       int* bad) {
  __shared__ long long d[kMaxParts];
  for (int p = threadIdx.x; p < k; p += kBlock) d[p] = 0;
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < n; v += stride) {
    const int p = label[v];
    if (p < 0 || p >= k) {
      *bad = 1;
      continue;
    }
    add_ll(&d[p], static_cast<long long>(weight ? weight[v] : 1));
  }
  __syncthreads();
  for (int p = threadIdx.x; p < k; p += kBlock)
    if (d[p] != 0) add_ll(&load[p], d[p]);
}

__global__ void __launch_bounds__(kBlock) k_add_delta(int k, long long* load,
                                                      const long long* delta) {
  if (threadIdx.x < k) load[threadIdx.x] += delta[threadIdx.x];
}

// cut edges of the in-CSR (edges whose endpoints sit in different parts)
__global__ void __launch_bounds__(kBlock) k_cut_edges(const int32_t* rows, const int32_t* idx,
                                                      int64_t nnz, const int32_t* label,
                                                      unsigned long long* cut) {
  unsigned long long c = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < nnz; j += stride)
    c += label[rows[j]] != label[idx[j]];
  // wave reduction then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cut, c);
}

__global__ void k_collect_heavy(const int32_t* in_ptr, const int32_t* out_ptr, int64_t n,
                                int32_t* heavy, unsigned long long* count) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < n; v += stride) {
    const int64_t d = (int64_t)(in_ptr[v + 1] - in_ptr[v]) + (out_ptr[v + 1] - out_ptr[v]);
    if (d >= kHeavy) heavy[atomicAdd(count, 1ull)] = static_cast<int32_t>(v);
  }
}

unsigned grid_for(int64_t items, int64_t per_block) {
  int64_t b = (items + per_block - 1) / per_block;
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(b, 65536)));
}

struct Fail : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Fail(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

extern "C" int DGLMIPartitionLabelProp(const DGLMIGraph* graph, int32_t num_parts, int32_t rounds,
                                       double slack, const int32_t* node_weight, uint64_t seed,
                                       int32_t* assign, int64_t* part_loads,
                                       int64_t* cut_edges, void* stream) {
  try {
    if (graph == nullptr || assign == nullptr) throw Fail("null argument");
    if (graph->num_bits != 32) throw Fail("partitioning needs int32 CSRs");
    if (num_parts < 1 || num_parts > kMaxParts)
      throw Fail("num_parts must be in [1, " + std::to_string(kMaxParts) + "]");
    if (rounds < 0) throw Fail("rounds must be >= 0");
    const DGLMICsr& ic = graph->in_csr;
    const DGLMICsr& oc = graph->out_csr;
    if (ic.num_rows != oc.num_rows || ic.num_rows != ic.num_cols)
      throw Fail("partitioning needs a square graph (num_src == num_dst)");
    if (ic.nnz > 0 && (!ic.indptr || !ic.indices || !ic.rows || !oc.indptr || !oc.indices))
      throw Fail("the graph needs in/out indptr, indices and the in-CSR rows");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t n = ic.num_rows;
    const int k = num_parts;
    // scratch: want (n), heavy list (n), two k x 256 histograms, loads / deltas /
    // cuts / rooms (k each), counters
    // released on every path out of here, the throwing ones included
    struct AsyncBuf {
      char* p = nullptr;
      hipStream_t s = nullptr;
      ~AsyncBuf() { if (p) (void)hipFreeAsync(p, s); }
    } buf;
    buf.s = s;
    const size_t want_b = ((n * sizeof(int32_t)) + 255) & ~size_t(255);
    const size_t hist_b = 2 * kMaxParts * 256 * sizeof(unsigned long long);
    const size_t small_b = 6 * kMaxParts * sizeof(long long) + 256;
    ck(hipMallocAsync(reinterpret_cast<void**>(&buf.p), 2 * want_b + hist_b + small_b, s),
       "hipMallocAsync");
    char* ws = buf.p;
    int32_t* want = reinterpret_cast<int32_t*>(ws);
    int32_t* heavy = reinterpret_cast<int32_t*>(ws + want_b);
    unsigned long long* hist_a = reinterpret_cast<unsigned long long*>(ws + 2 * want_b);
    unsigned long long* hist_bb = hist_a + kMaxParts * 256;
    long long* load = reinterpret_cast<long long*>(ws + 2 * want_b + hist_b);
    long long* delta = load + kMaxParts;
    long long* rem_a = delta + kMaxParts;
    long long* rem_b = rem_a + kMaxParts;
    int32_t* cut_a = reinterpret_cast<int32_t*>(rem_b + kMaxParts);
    int32_t* cut_b = cut_a + kMaxParts;
    unsigned long long* misc = reinterpret_cast<unsigned long long*>(cut_b + kMaxParts);
    // misc: [0] heavy count, [1] cut edges, [2] bad-label flag
    ck(hipMemsetAsync(load, 0, small_b, s), "hipMemsetAsync");
    hipLaunchKernelGGL(k_part_loads, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, k, assign,
                       node_weight, load, reinterpret_cast<int*>(&misc[2]));
    hipLaunchKernelGGL(k_collect_heavy, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, ic.indptr,
                       oc.indptr, n, heavy, &misc[0]);
    unsigned long long host_misc[3] = {0, 0, 0};
    long long host_load[kMaxParts];
    ck(hipMemcpyAsync(host_misc, misc, sizeof(host_misc), hipMemcpyDeviceToHost, s), "copy");
    ck(hipMemcpyAsync(host_load, load, k * sizeof(long long), hipMemcpyDeviceToHost, s), "copy");
    ck(hipStreamSynchronize(s), "sync");
    if (host_misc[2]) throw Fail("initial assignment holds a part id outside [0, num_parts)");
    const int64_t num_heavy = static_cast<int64_t>(host_misc[0]);
    long long total = 0;
    for (int p = 0; p < k; ++p) total += host_load[p];
    const long long cap =
        static_cast<long long>((1.0 + slack) * static_cast<double>(total) / k) + 1;
    LpArgs a{ic.indptr, ic.indices, oc.indptr, oc.indices, n, k, assign, node_weight, load,
             0, seed, want, hist_a};
    for (int r = 0; r < rounds && k > 1; ++r) {
      a.round = r;
      ck(hipMemsetAsync(hist_a, 0, hist_b, s), "memset");
      ck(hipMemsetAsync(delta, 0, kMaxParts * sizeof(long long), s), "memset");
      hipLaunchKernelGGL(k_lp_score_light, dim3(grid_for(n, kGroupsPerBlock)), dim3(kBlock), 0, s,
                         a);
      if (num_heavy > 0)
        hipLaunchKernelGGL(k_lp_score_heavy, dim3(grid_for(num_heavy, 1)), dim3(kBlock), 0, s, a,
                           heavy, num_heavy);
      hipLaunchKernelGGL(k_admit_cut, dim3(1), dim3(kMaxParts), 0, s, k, hist_a,
                         static_cast<const long long*>(nullptr), static_cast<const int32_t*>(nullptr),
                         cut_a, rem_a, load, cap);
      hipLaunchKernelGGL(k_admit_hist_b, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, want,
                         node_weight, r, seed, cut_a, hist_bb);
      hipLaunchKernelGGL(k_admit_cut, dim3(1), dim3(kMaxParts), 0, s, k, hist_bb, rem_a, cut_a,
                         cut_b, rem_b, load, cap);
      hipLaunchKernelGGL(k_lp_apply, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, k, want,
                         assign, node_weight, cut_a, cut_b, r, seed, delta);
      hipLaunchKernelGGL(k_add_delta, dim3(1), dim3(kMaxParts), 0, s, k, load, delta);
    }
    ck(hipGetLastError(), "launch");
    if (cut_edges) {
      hipLaunchKernelGGL(k_cut_edges, dim3(grid_for(ic.nnz, kBlock * 4)), dim3(kBlock), 0, s,
                         ic.rows, ic.indices, ic.nnz, assign, &misc[1]);
      ck(hipMemcpyAsync(host_misc, misc, sizeof(host_misc), hipMemcpyDeviceToHost, s), "copy");
    }
    if (part_loads)
      ck(hipMemcpyAsync(host_load, load, k * sizeof(long long), hipMemcpyDeviceToHost, s), "copy");
    (void)hipFreeAsync(buf.p, s);
    buf.p = nullptr;
    ck(hipStreamSynchronize(s), "sync");
    if (cut_edges) *cut_edges = static_cast<int64_t>(host_misc[1]);
    if (part_loads)
      for (int p = 0; p < k; ++p) part_loads[p] = host_load[p];
    return 0;
  } catch (const std::exception& e) {
    dglmi::set_last_error(e.what());
    return -1;
  }
}
