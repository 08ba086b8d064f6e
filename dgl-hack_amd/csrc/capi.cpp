// C ABI of the engine: validation, shape / broadcast inference, target -> role
// resolution and kernel dispatch.  Mirrors the reference dispatcher
// src/kernel/binary_reduce.cc (BinaryOpReduce :295-336, the Backward*
// variants :452-626, CopyReduce :628-716) and the device-agnostic drivers of
// src/kernel/binary_reduce_impl.h, with the reference's CHECK/LOG(FATAL)
// failures turned into -1 + DGLMIGetLastError() (runtime_base.h:13-32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "internal.h"

using namespace dglmi;

namespace {

thread_local std::string g_last_error;

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define DGLMI_CHECK(cond, msg)                                                     \
  do {                                                                             \
    if (!(cond)) throw Error(std::string("Check failed: " #cond ": ") + (msg));   \
  } while (0)

#define API_BEGIN() try {
#define API_END()                                 \
  }                                               \
  catch (const std::exception& e) {               \
    g_last_error = e.what();                      \
    return -1;                                    \
  }                                               \
  return 0;

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    check_hip(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) check_hip(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

int parse_reducer(const char* s) {
  DGLMI_CHECK(s != nullptr, "null reducer");
  const std::string r(s);
  if (r == "sum") return RED_SUM;
  if (r == "max") return RED_MAX;
  if (r == "min") return RED_MIN;
  if (r == "prod") return RED_PROD;
  if (r == "none") return RED_NONE;
  if (r == "mean") throw Error("reduce mean is not supported.");  // binary_reduce_impl.h:95-98
  throw Error("Unsupported reducer: " + r);
}

int parse_op(const char* s) {
  DGLMI_CHECK(s != nullptr, "null op");
  const std::string o(s);
  if (o == "add") return OP_ADD;
  if (o == "sub") return OP_SUB;
  if (o == "mul") return OP_MUL;
  if (o == "div") return OP_DIV;
  if (o == "dot") return OP_DOT;
  if (o == "use_lhs") return OP_USE_LHS;
  throw Error("Unsupported binary op: " + o);
}

std::string shape_str(const DGLMIArray* a) {
  std::string s = "(";
  for (int i = 1; i < a->ndim; ++i) {
    s += std::to_string(a->shape[i]);
    if (i + 1 < a->ndim) s += ",";
  }
  return s + ")";
}

int64_t feat_numel(const DGLMIArray* a) {
  int64_t n = 1;
  for (int i = 1; i < a->ndim; ++i) n *= a->shape[i];
  return n;
}

void check_array(const DGLMIArray* a, const char* name) {
  if (a == nullptr) throw Error(std::string("null array: ") + name);
  if (a->ndim < 1 || a->ndim > DGLMI_MAX_NDIM + 1)
    throw Error(std::string("bad ndim for ") + name);
  int64_t n = 1;
  for (int i = 0; i < a->ndim; ++i) {
    if (a->shape[i] < 0) throw Error(std::string("negative dim in ") + name);
    n *= a->shape[i];
  }
  if (n > 0 && a->data == nullptr) throw Error(std::string("null data pointer for ") + name);
}

// binary_reduce.cc:54-66
bool valid_elementwise(const DGLMIArray* l, const DGLMIArray* r) {
  if (l->ndim != r->ndim) return false;
  for (int i = 1; i < l->ndim; ++i)
    if (l->shape[i] != r->shape[i]) return false;
  return true;
}
// binary_reduce.cc:73-84
bool has_bcast(const DGLMIArray* l, const DGLMIArray* r) { return !valid_elementwise(l, r); }

// CalcBcastInfo (binary_reduce.cc:96-155).  real_out receives the feature
// shape the op produces (dot: including the vector length as the last dim).
Bcast calc_bcast(int op, const DGLMIArray* lhs, const DGLMIArray* rhs, std::vector<int64_t>* real_out) {
  Bcast b;
  std::memset(&b, 0, sizeof(b));
  std::vector<int64_t> ls, rs, os, ro;
  const int max_ndim = std::max(lhs->ndim, rhs->ndim) - 1;
  int64_t accum = 0;
  int j = 0;
  if (op == OP_DOT) {
    b.data_len = lhs->shape[lhs->ndim - 1];
    DGLMI_CHECK(rhs->shape[rhs->ndim - 1] == b.data_len, "dot operands differ in vector length");
    ++j;
    ro.push_back(b.data_len);
  } else {
    b.data_len = 1;
  }
  for (; j < max_ndim; ++j) {
    const int64_t dl = (lhs->ndim - 1 - j < 1) ? 1 : lhs->shape[lhs->ndim - 1 - j];
    const int64_t dr = (rhs->ndim - 1 - j < 1) ? 1 : rhs->shape[rhs->ndim - 1 - j];
    if (dl != dr) {
      if (dl != 1 && dr != 1)
        throw Error("Invalid broadcasting between feature shapes " + shape_str(lhs) + " and " +
                    shape_str(rhs));
      if (accum != 0) {
        ls.push_back(accum);
        rs.push_back(accum);
        os.push_back(accum);
        accum = 0;
      }
      ls.push_back(dl);
      rs.push_back(dr);
      os.push_back(std::max(dl, dr));
    } else {
      accum = accum == 0 ? dl : accum * dl;
    }
    ro.push_back(std::max(dl, dr));
  }
  if (accum != 0) {
    ls.push_back(accum);
    rs.push_back(accum);
    os.push_back(accum);
  }
  if (os.size() > static_cast<size_t>(kMaxDim)) throw Error("Too many broadcasting dimensions.");
  std::reverse(ro.begin(), ro.end());
  std::reverse(ls.begin(), ls.end());
  std::reverse(rs.begin(), rs.end());
  std::reverse(os.begin(), os.end());
  b.ndim = static_cast<int>(os.size());
  b.lhs_len = b.rhs_len = b.out_len = 1;
  for (int d = b.ndim - 1; d >= 0; --d) {
    b.lhs_shape[d] = ls[d];
    b.rhs_shape[d] = rs[d];
    b.out_shape[d] = os[d];
    b.lhs_stride[d] = (d == b.ndim - 1) ? 1 : b.lhs_stride[d + 1] * ls[d + 1];
    b.rhs_stride[d] = (d == b.ndim - 1) ? 1 : b.rhs_stride[d + 1] * rs[d + 1];
    b.out_stride[d] = (d == b.ndim - 1) ? 1 : b.out_stride[d + 1] * os[d + 1];
    b.lhs_len *= ls[d];
    b.rhs_len *= rs[d];
    b.out_len *= os[d];
  }
  if (real_out) *real_out = ro;
  return b;
}

// 32: every index array int32 (the reference GPU envelope, common.h:62-69); 64: a
// graph of 2^31 or more edges, whose indptr and data (edge ids) hold int64 -- the
// width the reference's CPU kernels switch to (graph_index.py:941-952,
// cpu/binary_reduce_sum.cc:15-23) -- while node ids (indices, rows, COO) stay int32.
void check_graph(const DGLMIGraph* g) {
  DGLMI_CHECK(g != nullptr, "null graph");
  if (g->num_bits != 32 && g->num_bits != 64)
    throw Error("Unsupported idx bits: " + std::to_string(g->num_bits));
}

// Entry points built for int32 graphs only (the hack's kernels are int32-only,
// binary_reduce_impl.cu: typedef int32_t Idx).
void check_graph32(const DGLMIGraph* g, const char* what) {
  check_graph(g);
  if (g->num_bits != 32)
    throw Error(std::string(what) + " needs a graph of fewer than 2^31 edges (idx bits 32)");
}

bool wide(const DGLMIGraph* g) { return g->num_bits == 64; }

IdxPtr idx(const DGLMIGraph* g, const int32_t* p) { return IdxPtr{p, wide(g) ? 1 : 0}; }

void check_csr(const DGLMICsr& c, const char* which, bool need_rows, bool wide_ok = false) {
  if (c.num_rows < 0 || c.nnz < 0) throw Error(std::string("bad CSR sizes: ") + which);
  if (c.indptr == nullptr) throw Error(std::string("null indptr: ") + which);
  if (c.nnz > 0 && (c.indices == nullptr || c.data == nullptr))
    throw Error(std::string("null CSR arrays: ") + which);
  if (need_rows && c.nnz > 0 && c.rows == nullptr)
    throw Error(std::string("CSR row ids (rows) required: ") + which);
  if (c.num_rows > INT32_MAX || c.num_cols > INT32_MAX)
    throw Error("graph exceeds int32 node ids");
  if (!wide_ok && c.nnz > INT32_MAX)
    throw Error("graph exceeds int32 indexing (2^31 or more edges need idx bits 64)");
}

// Mappings index by edge id and name rows of int32 range: not for 64-bit graphs.
void check_maps(const DGLMIGraph* g, const int32_t* a, const int32_t* b, const int32_t* c) {
  if (wide(g) && (a || b || c))
    throw Error("node / edge mappings need a graph of fewer than 2^31 edges (idx bits 32)");
}

int role_of(int target, bool walk_in) {
  // in-CSR: row = dst, col = src ; out-CSR: row = src, col = dst
  switch (target) {
    case DGLMI_TARGET_SRC: return walk_in ? ROLE_COL : ROLE_ROW;
    case DGLMI_TARGET_DST: return walk_in ? ROLE_ROW : ROLE_COL;
    case DGLMI_TARGET_EDGE: return ROLE_EDGE;
    default: return ROLE_NONE;
  }
}

float identity_of(int red) {
  switch (red) {
    case RED_MAX: return -3.402823466e+38f;
    case RED_MIN: return 3.402823466e+38f;
    case RED_PROD: return 1.0f;
    default: return 0.0f;
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Scratch for the load-balanced path: the caller's workspace, or a
// stream-ordered allocation released on the same stream.
// Keep stream-ordered scratch in the device's default pool between calls: with
// the default release threshold (0) every synchronisation hands the pool's
// memory back and the next call maps it again (hundreds of MB for the blocked
// GAT partials).  The engine's own allocations are the only users of the pool
// (torch has its caching allocator), so the pool's size stays at the largest
// scratch a call needed.
void keep_pool_memory() {
  static bool done[64] = {false};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || done[dev]) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t thr = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  done[dev] = true;
}

struct Scratch {
  void* ptr = nullptr;
  bool owned = false;
  hipStream_t s = nullptr;
  Scratch(const DGLMIGraph* g, int64_t bytes, hipStream_t stream) : s(stream) {
    if (bytes <= 0) return;
    if (g->workspace != nullptr && g->workspace_bytes >= bytes) {
      ptr = g->workspace;
    } else {
      keep_pool_memory();
      check_hip(hipMallocAsync(&ptr, static_cast<size_t>(bytes), stream), "hipMallocAsync");
      owned = true;
    }
  }
  ~Scratch() {
    if (owned && ptr) (void)hipFreeAsync(ptr, s);
  }
};

// Run a reduce-to-row on the load-balanced kernels.  `walk` is the CSR whose
// rows own the output; out has `walk.num_rows` rows of F floats.
void run_fast(const DGLMIGraph* g, const DGLMICsr& walk, int kind, int red, const float* x,
              const int32_t* x_map, const float* w, const int32_t* w_map, float* out, int64_t F,
              int64_t head_dim, hipStream_t s, const DGLMIEpilogue* epi = nullptr,
              const float* xr = nullptr);

// Column blocks (DGLMIGraph.num_col_blocks) on the load-balanced sum: one pass
// per non-empty block, so a pass gathers from a slice of the table that fits the
// 4 MiB per-XCD L2; the partial sums chain through the epilogue's addend
// (ping-pong between `out` and a scratch buffer, the last pass lands in `out`).
// Every pass applies row_mul / row_div to its own sum (sum_b acc_b * m / d ==
// (sum_b acc_b) * m / d up to rounding); the caller's addend enters with the
// first pass, the bias with the last.  Block order is fixed: deterministic.
void run_fast_blocked(const DGLMIGraph* g, const DGLMICsr* blocks, const DGLMICsr& walk, int kind,
                      const float* x, const float* w, const int32_t* w_map, float* out, int64_t F,
                      int64_t head_dim, hipStream_t s, const DGLMIEpilogue* epi) {
  std::vector<int> nz;
  for (int b = 0; b < g->num_col_blocks; ++b) {
    DGLMI_CHECK(blocks[b].num_rows == walk.num_rows && blocks[b].indptr != nullptr,
                "column blocks must keep the graph's rows");
    if (blocks[b].nnz > 0) nz.push_back(b);
  }
  DGLMIGraph plain = *g;  // no blocks / hints for the per-block passes
  plain.num_col_blocks = 0;
  plain.in_col_blocks = plain.out_col_blocks = nullptr;
  plain.in_gather_cols = plain.out_gather_cols = nullptr;
  if (nz.size() <= 1) {
    run_fast(&plain, nz.empty() ? walk : blocks[nz[0]], kind, RED_SUM, x, nullptr, w, w_map, out, F,
             head_dim, s, epi);
    return;
  }
  DGLMIGraph no_ws;  // the ping-pong buffer must not alias the carry workspace
  std::memset(&no_ws, 0, sizeof(no_ws));
  Scratch tmp(&no_ws, walk.num_rows * F * static_cast<int64_t>(sizeof(float)), s);
  float* bufs[2] = {out, static_cast<float*>(tmp.ptr)};
  const int k = static_cast<int>(nz.size());
  const float* prev = epi ? epi->addend : nullptr;
  for (int i = 0; i < k; ++i) {
    float* dst = bufs[(k - 1 - i) % 2];
    DGLMIEpilogue e;
    e.row_mul = epi ? epi->row_mul : nullptr;
    e.row_div = epi ? epi->row_div : nullptr;
    e.bias = (epi && i == k - 1) ? epi->bias : nullptr;
    e.addend = prev;
    const bool any = e.row_mul || e.row_div || e.bias || e.addend;
    run_fast(&plain, blocks[nz[i]], kind, RED_SUM, x, nullptr, w, w_map, dst, F, head_dim, s,
             any ? &e : nullptr);
    prev = dst;
  }
}

void run_fast(const DGLMIGraph* g, const DGLMICsr& walk, int kind, int red, const float* x,
              const int32_t* x_map, const float* w, const int32_t* w_map, float* out, int64_t F,
              int64_t head_dim, hipStream_t s, const DGLMIEpilogue* epi, const float* xr) {
  // copy_u only: with an edge operand (u_mul_e) its per-edge gather by edge id
  // dominates and extra passes cost more than the smaller table saves (Reddit-size,
  // F = 64: copy_u_sum 3.88 -> 2.96 ms over 8 blocks, u_mul_e_sum 5.94 -> 7.23 ms)
  if (g->num_col_blocks > 1 && !wide(g) && red == RED_SUM && x_map == nullptr && walk.nnz > 0 &&
      kind == FAST_COPY_COL) {
    const DGLMICsr* blocks = &walk == &g->in_csr ? g->in_col_blocks
                             : (&walk == &g->out_csr ? g->out_col_blocks : nullptr);
    if (blocks != nullptr) {
      run_fast_blocked(g, blocks, walk, kind, x, w, w_map, out, F, head_dim, s, epi);
      return;
    }
  }
  if (walk.nnz == 0) {
    launch_fill(out, walk.num_rows * F, identity_of(red), s);
    if (epi) launch_epilogue(out, walk.num_rows, F, epi->row_mul, epi->row_div, epi->bias, epi->addend, s);
    return;
  }
  FastArgs a;
  std::memset(&a, 0, sizeof(a));
  a.indptr = idx(g, walk.indptr);
  a.rows = walk.rows;
  a.indices = walk.indices;
  // a position view's walk (DGLMIGraph.eid_identity), or an internal walk whose edge
  // ids are its positions (data NULL: the R-GCN state's position-ordered walks): edge
  // p's operand sits at p
  const int id_bit = &walk == &g->in_csr ? 1 : (&walk == &g->out_csr ? 2 : 0);
  a.eids = ((g->eid_identity & id_bit) != 0 || walk.data == nullptr) ? IdxPtr{nullptr, wide(g) ? 1 : 0}
                                                                      : idx(g, walk.data);
  a.nnz = walk.nnz;
  a.num_rows = walk.num_rows;
  a.x = x;
  a.w = w;
  a.x_map = x_map;
  a.w_map = w_map;
  a.out = out;
  a.F = F;
  a.head_dim = head_dim;
  a.chunk = fast_chunk_edges(walk.nnz, F);
  a.xr = xr;
  // cold-row hints: copy_u sum over a table larger than the Infinity Cache
  if (kind == FAST_COPY_COL && red == RED_SUM && x_map == nullptr && fast_marked_supported(F)) {
    const int32_t* marked = &walk == &g->in_csr ? g->in_gather_cols
                            : (&walk == &g->out_csr ? g->out_gather_cols : nullptr);
    if (marked != nullptr && walk.num_cols * F * static_cast<int64_t>(sizeof(float)) >= kMarkedMinTableBytes) {
      a.indices = marked;
      a.marked = 1;
      a.num_cols = walk.num_cols;
    }
  }
  if (epi) {
    a.row_mul = epi->row_mul;
    a.row_div = epi->row_div;
    a.bias = epi->bias;
    a.addend = epi->addend;
  }
  // one weight per edge, read at the position: staged with the walk (FAST_COL_MUL_POS)
  if (kind == FAST_COL_MUL_EDGE_BCAST && !a.eids && head_dim == F && w_map == nullptr &&
      red == RED_SUM)
    kind = FAST_COL_MUL_POS;
  Scratch carry(g, fast_workspace_bytes(walk.nnz, F), s);
  a.carry = static_cast<float*>(carry.ptr);
  a.seg_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(carry.ptr) + fast_carry_bytes(walk.nnz, F));
  launch_fast_reduce(kind, red, a, s);
  check_hip(hipGetLastError(), "fast reduce launch");
}

// Items of a per-edge kernel.  Edge-id order (the graph's COO) streams the
// output and any edge operand sequentially and gathers both node rows; in-CSR
// order keeps the destination row in cache along its run but scatters the
// output by eid.  Measured (scripts/bench_configs.py sd, scripts/
// sddmm_order_probe.py): on M1 (average in-degree 12) edge-id order wins even
// for wide node-only ops (u_dot_v F = 64: 6.07 vs 7.28 ms) and by far for
// narrow rows (u_add_v H = 8: 3.66 vs 5.25 ms); on the Reddit-size graph
// (average in-degree 492) in-CSR order wins for wide node-only rows (u_dot_v
// 8 x 8: 7.38 vs 8.10 ms) while narrow rows still prefer edge-id order (3.64 vs
// 5.55 ms).  So: in-CSR order only for node-only operands, rows of >= 32
// floats and average in-degree >= 64.  DGLMISetSddmmOrder forces one (tests
// of both walks, scripts/sddmm_order_probe.py).
std::atomic<int> g_sddmm_order{DGLMI_SDDMM_ORDER_AUTO};

SddmmArgs sddmm_items(const DGLMIGraph* g, const DGLMICsr& walk, bool edge_operand,
                      int64_t row_floats) {
  SddmmArgs e;
  std::memset(&e, 0, sizeof(e));
  e.nnz = walk.nnz;
  bool coo = g->coo_src != nullptr && g->coo_dst != nullptr;
  if (coo) {
    const int forced = g_sddmm_order.load(std::memory_order_relaxed);
    if (forced == DGLMI_SDDMM_ORDER_CSR) coo = false;
    else if (forced != DGLMI_SDDMM_ORDER_COO)
      coo = edge_operand || row_floats < 32 || walk.nnz < 64 * std::max<int64_t>(walk.num_rows, 1);
  }
  if (coo) {
    e.rows = g->coo_dst;
    e.cols = g->coo_src;
    e.eids = IdxPtr{nullptr, 0};
  } else {
    e.rows = walk.rows;
    e.cols = walk.indices;
    e.eids = idx(g, walk.data);
  }
  return e;
}

EdgeArgs base_args(const DGLMIGraph* g, const DGLMICsr& walk) {
  EdgeArgs a;
  std::memset(&a, 0, sizeof(a));
  a.indptr = idx(g, walk.indptr);
  a.indices = walk.indices;
  a.eids = idx(g, walk.data);
  a.rows = walk.rows;
  a.num_rows = walk.num_rows;
  a.nnz = walk.nnz;
  a.len = 1;
  return a;
}

// ---------------------------------------------------------------------------
// Forward: BinaryOpReduce / CopyReduce
// ---------------------------------------------------------------------------
void forward(int red, int op, const DGLMIGraph* g, int lhs_t, int rhs_t, const DGLMIArray* lhs,
             const DGLMIArray* rhs, DGLMIArray* out, const int32_t* lhs_map,
             const int32_t* rhs_map, const int32_t* out_map, hipStream_t s,
             const DGLMIEpilogue* epi = nullptr) {
  if (epi && !epi->row_mul && !epi->row_div && !epi->bias && !epi->addend) epi = nullptr;
  DGLMI_CHECK(epi == nullptr || red == RED_SUM, "a fused epilogue needs the sum reducer");
  check_graph(g);
  check_maps(g, lhs_map, rhs_map, out_map);
  check_array(lhs, "lhs");
  check_array(out, "out");
  DGLMI_CHECK(lhs_t >= 0 && lhs_t <= 2, "bad lhs target");
  if (op != OP_USE_LHS) {
    check_array(rhs, "rhs");
    DGLMI_CHECK(rhs_t >= 0 && rhs_t <= 2, "bad rhs target");
    DGLMI_CHECK(lhs_t != rhs_t, "lhs and rhs targets must differ");  // binary_reduce.cc:216
    if ((op == OP_ADD || op == OP_MUL) && lhs_t > rhs_t) {  // NeedSwitchOrder :214-219
      std::swap(lhs_t, rhs_t);
      std::swap(lhs, rhs);
      std::swap(lhs_map, rhs_map);
    }
  }
  const DGLMICsr& walk = g->in_csr;  // reductions go to dst; edges enumerated on the in-CSR
  check_csr(walk, "in_csr", red == RED_NONE || true, wide(g));

  bool bc = false;
  Bcast binfo;
  std::memset(&binfo, 0, sizeof(binfo));
  int64_t D, len = 1;
  if (op == OP_USE_LHS) {
    D = feat_numel(lhs);
  } else if (has_bcast(lhs, rhs)) {
    bc = true;
    binfo = calc_bcast(op, lhs, rhs, nullptr);
    D = binfo.out_len;
    len = binfo.data_len;
  } else {
    if (!valid_elementwise(lhs, rhs))
      throw Error("Cannot compute binary operation between feature shapes " + shape_str(lhs) +
                  " and " + shape_str(rhs));
    if (op == OP_DOT) {
      len = lhs->shape[lhs->ndim - 1];
      D = feat_numel(lhs) / std::max<int64_t>(len, 1);
      if (len == 0) D = 0;
    } else {
      D = feat_numel(lhs);
    }
  }
  DGLMI_CHECK(feat_numel(out) == D, "out feature size " + std::to_string(feat_numel(out)) +
                                        " != expected " + std::to_string(D));
  const int64_t out_rows = out->shape[0];
  const int64_t expect_rows = red == RED_NONE ? walk.nnz : walk.num_rows;
  const bool need_fill = out_map != nullptr || out_rows != expect_rows;
  if (!out_map) DGLMI_CHECK(out_rows >= expect_rows, "out has too few rows");
  if (out_rows * D == 0) return;

  // ---- load-balanced path for the hot reduce-to-dst message functions ----
  if (red != RED_NONE && out_map == nullptr && out_rows == walk.num_rows && red != RED_PROD &&
      aligned16(out->data) && aligned16(lhs->data)) {
    int kind = -1;
    int64_t head_dim = 1;
    if (op == OP_USE_LHS && lhs_t == DGLMI_TARGET_SRC) kind = FAST_COPY_COL;
    else if (op == OP_USE_LHS && lhs_t == DGLMI_TARGET_EDGE) kind = FAST_COPY_EDGE;
    else if (op == OP_MUL && red == RED_SUM && lhs_t == DGLMI_TARGET_SRC &&
             rhs_t == DGLMI_TARGET_EDGE && aligned16(rhs->data)) {
      if (!bc) {
        kind = FAST_COL_MUL_EDGE;
      } else if (binfo.ndim == 2 && binfo.rhs_shape[1] == 1 && binfo.lhs_shape[0] == binfo.rhs_shape[0] &&
                 binfo.lhs_shape[1] == binfo.out_shape[1]) {
        kind = FAST_COL_MUL_EDGE_BCAST;  // (N, H, D) x (E, H, 1): GAT aggregation
        head_dim = binfo.lhs_shape[1];
      } else if (binfo.ndim == 1 && binfo.rhs_shape[0] == 1) {
        kind = FAST_COL_MUL_EDGE_BCAST;  // (N, D) x (E, 1)
        head_dim = binfo.lhs_shape[0];
      }
    }
    if (kind >= 0 && fast_supported(kind, D, head_dim) && walk.rows != nullptr) {
      const float* w = (kind == FAST_COL_MUL_EDGE || kind == FAST_COL_MUL_EDGE_BCAST) ? rhs->data : nullptr;
      const bool epi_ok = epi == nullptr || ((epi->bias == nullptr || aligned16(epi->bias)) &&
                                             (epi->addend == nullptr || aligned16(epi->addend)));
      if (epi_ok) {
        run_fast(g, walk, kind, red, lhs->data, lhs_map, w, rhs_map, out->data, D, head_dim, s, epi);
        return;
      }
    }
  }

  if (need_fill) launch_fill(out->data, out_rows * D, identity_of(red), s);
  if (red == RED_NONE && walk.nnz > 0) DGLMI_CHECK(walk.rows != nullptr, "in_csr.rows required");

  // ---- per-edge outputs (g-SDDMM) ----
  if (red == RED_NONE && !bc && !lhs_map && !rhs_map && !out_map && walk.nnz > 0 &&
      sddmm_supported(op == OP_DOT && len == 1 ? OP_MUL : op, false, D, len) &&
      aligned16(out->data) && aligned16(lhs->data) && (op == OP_USE_LHS || aligned16(rhs->data))) {
    SddmmArgs e = sddmm_items(g, walk, lhs_t == DGLMI_TARGET_EDGE ||
                                           (op != OP_USE_LHS && rhs_t == DGLMI_TARGET_EDGE),
                              D * len);
    e.lhs = lhs->data;
    e.lhs_role = role_of(lhs_t, true);
    e.rhs = op == OP_USE_LHS ? nullptr : rhs->data;
    e.rhs_role = op == OP_USE_LHS ? ROLE_NONE : role_of(rhs_t, true);
    e.out = out->data;
    e.D = D;
    e.len = len;
    launch_sddmm(op == OP_DOT && len == 1 ? OP_MUL : op, false, e, s);
    check_hip(hipGetLastError(), "sddmm launch");
    return;
  }

  // ---- generic path (load-balanced for reductions) ----
  EdgeArgs a = base_args(g, walk);
  a.lhs = Operand{lhs->data, lhs_map, role_of(lhs_t, true)};
  if (op == OP_USE_LHS) a.rhs = Operand{nullptr, nullptr, ROLE_NONE};
  else a.rhs = Operand{rhs->data, rhs_map, role_of(rhs_t, true)};
  a.out = out->data;
  a.out_map = out_map;
  a.out_role = red == RED_NONE ? ROLE_EDGE : ROLE_ROW;
  a.D = D;
  a.len = len;
  a.out_rows = out_rows;
  a.bc = binfo;
  if (red != RED_NONE && walk.rows != nullptr && generic_lb_supported(D)) {
    if (walk.nnz == 0) {
      if (!need_fill) launch_fill(out->data, walk.num_rows * D, identity_of(red), s);
      if (epi) launch_epilogue(out->data, out_rows, D, epi->row_mul, epi->row_div, epi->bias, epi->addend, s);
      return;
    }
    a.chunk = fast_chunk_edges(walk.nnz, D);
    Scratch carry(g, fast_workspace_bytes(walk.nnz, D), s);
    a.carry = static_cast<float*>(carry.ptr);
    a.seg_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(carry.ptr) + fast_carry_bytes(walk.nnz, D));
    launch_generic_lb(op, red, bc, false, a, s);
    check_hip(hipGetLastError(), "generic lb forward launch");
    if (epi) launch_epilogue(out->data, out_rows, D, epi->row_mul, epi->row_div, epi->bias, epi->addend, s);
    return;
  }
  launch_generic_forward(op, red, bc, a, s);
  check_hip(hipGetLastError(), "generic forward launch");
  if (epi) launch_epilogue(out->data, out_rows, D, epi->row_mul, epi->row_div, epi->bias, epi->addend, s);
}

// ---------------------------------------------------------------------------
// Backward: Backward{Lhs,Rhs}BinaryOpReduce / BackwardCopyReduce
// ---------------------------------------------------------------------------
void backward(int red, int op, const DGLMIGraph* g, int lhs_t, int rhs_t, const int32_t* lhs_map,
              const int32_t* rhs_map, const int32_t* out_map, const DGLMIArray* lhs,
              const DGLMIArray* rhs, const DGLMIArray* out, const DGLMIArray* grad_out,
              DGLMIArray* grad, int want, hipStream_t s) {
  check_graph(g);
  check_maps(g, lhs_map, rhs_map, out_map);
  check_array(lhs, "lhs");
  check_array(out, "out");
  check_array(grad_out, "grad_out");
  check_array(grad, "grad");
  DGLMI_CHECK(lhs_t >= 0 && lhs_t <= 2, "bad lhs target");
  if (op != OP_USE_LHS) {
    check_array(rhs, "rhs");
    DGLMI_CHECK(rhs_t >= 0 && rhs_t <= 2, "bad rhs target");
    DGLMI_CHECK(lhs_t != rhs_t, "lhs and rhs targets must differ");
    if ((op == OP_ADD || op == OP_MUL) && lhs_t > rhs_t) {  // binary_reduce.cc:470-476, 571-577
      std::swap(lhs_t, rhs_t);
      std::swap(lhs, rhs);
      std::swap(lhs_map, rhs_map);
      want = 1 - want;
    }
  } else {
    DGLMI_CHECK(want == 0, "copy reduce has no rhs gradient");
  }
  const int x_t = want == 0 ? lhs_t : rhs_t;
  const bool walk_in = x_t != DGLMI_TARGET_SRC;  // src grads are owned by out-CSR rows
  const DGLMICsr& walk = walk_in ? g->in_csr : g->out_csr;
  check_csr(walk, walk_in ? "in_csr" : "out_csr", x_t == DGLMI_TARGET_EDGE, wide(g));

  bool bc = false;
  Bcast binfo;
  std::memset(&binfo, 0, sizeof(binfo));
  int64_t D, len = 1;
  if (op == OP_USE_LHS) {
    D = feat_numel(lhs);
  } else if (has_bcast(lhs, rhs)) {
    bc = true;
    binfo = calc_bcast(op, lhs, rhs, nullptr);
    D = binfo.out_len;
    len = binfo.data_len;
  } else {
    if (!valid_elementwise(lhs, rhs))
      throw Error("Cannot compute binary operation between feature shapes " + shape_str(lhs) +
                  " and " + shape_str(rhs));
    len = op == OP_DOT ? lhs->shape[lhs->ndim - 1] : 1;
    D = op == OP_DOT ? (len ? feat_numel(lhs) / len : 0) : feat_numel(lhs);
  }
  DGLMI_CHECK(feat_numel(out) == D && feat_numel(grad_out) == D, "out / grad_out feature size mismatch");
  const int64_t Dg = D * len;
  DGLMI_CHECK(feat_numel(grad) == Dg, "grad feature size " + std::to_string(feat_numel(grad)) +
                                          " != expected " + std::to_string(Dg));
  const int64_t grad_rows = grad->shape[0];
  if (grad_rows * Dg == 0) return;
  const int32_t* x_map = want == 0 ? lhs_map : rhs_map;
  const int64_t expect_rows = x_t == DGLMI_TARGET_EDGE ? walk.nnz : walk.num_rows;
  if (!x_map) DGLMI_CHECK(grad_rows >= expect_rows, "grad has too few rows");
  const bool need_fill = x_map != nullptr || grad_rows != expect_rows;

  // ---- load-balanced path: gradients that are themselves a reduce-to-row ----
  // copy_u_sum:  grad_u[src] = sum_{dst in out(src)} grad_out[dst]
  // u_mul_e_sum: grad_u[src] = sum grad_out[dst] * e[eid]  (the reference's
  // csrmm2-on-out-CSR specialisation, binary_reduce_sum.cu:262-292).
  if (red == RED_SUM && x_t == DGLMI_TARGET_SRC && !need_fill && out_map == nullptr &&
      walk.rows != nullptr && aligned16(grad->data) && aligned16(grad_out->data)) {
    int kind = -1;
    int64_t head_dim = 1;
    const float* w = nullptr;
    const int32_t* w_map = nullptr;
    if (op == OP_USE_LHS) {
      kind = FAST_COPY_COL;
    } else if (op == OP_MUL && want == 0 && rhs_t == DGLMI_TARGET_EDGE && aligned16(rhs->data)) {
      w = rhs->data;
      w_map = rhs_map;
      if (!bc) {
        kind = FAST_COL_MUL_EDGE;
      } else if (binfo.ndim == 2 && binfo.rhs_shape[1] == 1 && binfo.lhs_shape[0] == binfo.rhs_shape[0] &&
                 binfo.lhs_shape[1] == binfo.out_shape[1]) {
        kind = FAST_COL_MUL_EDGE_BCAST;
        head_dim = binfo.lhs_shape[1];
      } else if (binfo.ndim == 1 && binfo.rhs_shape[0] == 1) {
        kind = FAST_COL_MUL_EDGE_BCAST;
        head_dim = binfo.lhs_shape[0];
      }
    }
    if (kind >= 0 && fast_supported(kind, D, head_dim)) {
      run_fast(g, walk, kind, RED_SUM, grad_out->data, nullptr, w, w_map, grad->data, D, head_dim, s);
      return;
    }
  }

  // u_add_v / u_add_e / u_sub_v (lhs) with reducer none: a node operand's gradient is the
  // edge gradient summed over the node's walk row (binary_reduce_impl.cc's
  // BackwardBinaryReduce with the add/sub grad = grad_out), i.e. copy_e_sum on the walk
  // -- the load-balanced copy_e kernel, 16-B edge rows, instead of the generic
  // lane-per-feature walk (C3 GAT composition, H = 8: the two u_add_v gradients took
  // 3.35 + 2.65 ms there)
  if (red == RED_NONE && (op == OP_ADD || (op == OP_SUB && want == 0)) && !bc &&
      x_t != DGLMI_TARGET_EDGE && !need_fill && out_map == nullptr && walk.rows != nullptr &&
      aligned16(grad->data) && aligned16(grad_out->data) && fast_supported(FAST_COPY_EDGE, D, 1)) {
    run_fast(g, walk, FAST_COPY_EDGE, RED_SUM, grad_out->data, nullptr, nullptr, nullptr, grad->data,
             D, 1, s);
    return;
  }

  // copy_u max / min: grad_u[src] = sum over out-edges of grad_out[dst] where
  // x[src] == out[dst] (every tied edge, the reference's BackwardCall for max /
  // min) -- a reduce-to-row over the out-CSR with a tie-mask edge value, so the
  // load-balanced kernels own each source row (no atomics)
  if ((red == RED_MAX || red == RED_MIN) && op == OP_USE_LHS && x_t == DGLMI_TARGET_SRC &&
      !need_fill && out_map == nullptr && lhs_map == nullptr && walk.rows != nullptr &&
      aligned16(grad->data) && aligned16(grad_out->data) && aligned16(out->data) &&
      aligned16(lhs->data) && fast_supported(FAST_COL_TIE, D, 1)) {
    run_fast(g, walk, FAST_COL_TIE, RED_SUM, grad_out->data, nullptr, out->data, nullptr, grad->data,
             D, 1, s, nullptr, lhs->data);
    return;
  }

  if (need_fill) launch_fill(grad->data, grad_rows * Dg, 0.0f, s);

  // ---- per-edge gradients (g-SDDMM shape) for reducers none / sum ----
  if (x_t == DGLMI_TARGET_EDGE && (red == RED_NONE || red == RED_SUM) && !bc && !lhs_map &&
      !rhs_map && !out_map && walk.nnz > 0 && walk.rows != nullptr &&
      sddmm_supported(op == OP_DOT && len == 1 ? OP_MUL : op, true, D, len) &&
      aligned16(grad->data) && aligned16(grad_out->data) && aligned16(lhs->data) &&
      (op == OP_USE_LHS || aligned16(rhs->data))) {
    SddmmArgs e = sddmm_items(g, walk, true, Dg);  // a gradient row is an edge array
    e.lhs = lhs->data;
    e.lhs_role = role_of(lhs_t, true);
    e.rhs = op == OP_USE_LHS ? nullptr : rhs->data;
    e.rhs_role = op == OP_USE_LHS ? ROLE_NONE : role_of(rhs_t, true);
    e.out = grad->data;
    e.go = grad_out->data;
    e.go_role = red == RED_NONE ? ROLE_EDGE : ROLE_ROW;
    e.want = want;
    e.D = D;
    e.len = len;
    launch_sddmm(op == OP_DOT && len == 1 ? OP_MUL : op, true, e, s);
    check_hip(hipGetLastError(), "sddmm backward launch");
    return;
  }

  EdgeArgs a = base_args(g, walk);
  a.lhs = Operand{lhs->data, lhs_map, role_of(lhs_t, walk_in)};
  if (op == OP_USE_LHS) a.rhs = Operand{nullptr, nullptr, ROLE_NONE};
  else a.rhs = Operand{rhs->data, rhs_map, role_of(rhs_t, walk_in)};
  a.out = grad->data;
  a.out_role = x_t == DGLMI_TARGET_EDGE ? ROLE_EDGE : ROLE_ROW;
  a.D = D;
  a.len = len;
  a.out_rows = grad_rows;
  a.fwd_out = out->data;
  a.grad_out = grad_out->data;
  a.fo_map = out_map;
  a.fo_role = red == RED_NONE ? ROLE_EDGE : role_of(DGLMI_TARGET_DST, walk_in);
  a.want = want;
  a.bc = binfo;
  // node-owned gradients: load-balanced over CSR positions
  if (x_t != DGLMI_TARGET_EDGE && walk.rows != nullptr && generic_lb_supported(Dg)) {
    if (walk.nnz == 0) {
      if (!need_fill) launch_fill(grad->data, walk.num_rows * Dg, 0.0f, s);
      return;
    }
    a.chunk = fast_chunk_edges(walk.nnz, Dg);
    Scratch carry(g, fast_workspace_bytes(walk.nnz, Dg), s);
    a.carry = static_cast<float*>(carry.ptr);
    a.seg_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(carry.ptr) + fast_carry_bytes(walk.nnz, Dg));
    launch_generic_lb(op, red, bc, true, a, s);
    check_hip(hipGetLastError(), "generic lb backward launch");
    return;
  }
  launch_generic_backward(op, red, bc, a, s);
  check_hip(hipGetLastError(), "generic backward launch");
}

// Shared argument checking of the fused GAT entry points.
// Column blocks usable by the fused GAT kernels: every block non-empty (block 0
// of the destination-side walk must see every row) and shaped like the graph.
int gat_blocks(const DGLMIGraph* g) {
  const int nb = g->num_col_blocks;
  if (nb <= 1 || g->in_col_blocks == nullptr || g->out_col_blocks == nullptr) return 1;
  for (int b = 0; b < nb; ++b) {
    const DGLMICsr& i = g->in_col_blocks[b];
    const DGLMICsr& o = g->out_col_blocks[b];
    check_csr(i, "in_col_blocks", true);
    check_csr(o, "out_col_blocks", true);
    DGLMI_CHECK(i.num_rows == g->in_csr.num_rows && o.num_rows == g->out_csr.num_rows,
                "column blocks must keep the graph's rows");
    if (i.nnz == 0 || o.nnz == 0) return 1;
  }
  return nb;
}

// Chunk size of the backward walks: one halving beyond the forward's rule
// (gat_chunk_edges) while a launch would have fewer than 2 x 16 K groups.  On C3's
// column blocks (~14 M edges per launch) K = 512 leaves ~7000 waves per launch, and
// the two backward walks wait on memory ~60 % of their wave cycles (SQ_WAIT_ANY /
// SQ_WAVE_CYCLES, profiles/r03_gat_pmc_blocked.json); K = 256 hides more of it:
// backward 8.92 -> 8.45 ms, while the forward stays best at 512
// (profiles/r03_tune_gat_chunk.json).  Unblocked C3 (114 M edges) keeps 512.
int64_t gat_bwd_chunk_edges(int64_t nnz) {
  int64_t k = gat_chunk_edges(nnz);
  if (k > 8 && nnz / k < 2 * 256 * 64) k >>= 1;
  return k;
}

GatArgs gat_args(const DGLMIGraph* g, const DGLMIArray* ft, const DGLMIArray* el,
                 const DGLMIArray* er, float slope, DGLMIArray* out, DGLMIArray* mx,
                 DGLMIArray* sm) {
  check_array(ft, "feat_src");
  check_array(el, "el");
  check_array(er, "er");
  check_array(out, "out");
  check_array(mx, "max");
  check_array(sm, "sum");
  DGLMI_CHECK(ft->ndim == 3, "feat_src must be (N, H, D)");
  const int64_t H = ft->shape[1], D = ft->shape[2];
  if (!gat_supported(H, D))
    throw Error("fused GAT: unsupported heads/head_dim (" + std::to_string(H) + ", " +
                std::to_string(D) + "); D must be a multiple of 4 with D/4 a power of two");
  const DGLMICsr& in = g->in_csr;
  check_csr(in, "in_csr", true);
  DGLMI_CHECK(in.num_cols == ft->shape[0] || in.nnz == 0, "in_csr columns != feat_src rows");
  DGLMI_CHECK(el->shape[0] == ft->shape[0] && feat_numel(el) == H, "el must be (N_src, H[, 1])");
  DGLMI_CHECK(er->shape[0] == in.num_rows && feat_numel(er) == H, "er must be (N_dst, H[, 1])");
  DGLMI_CHECK(out->shape[0] == in.num_rows && feat_numel(out) == H * D, "out must be (N_dst, H, D)");
  DGLMI_CHECK(mx->shape[0] == in.num_rows && feat_numel(mx) == H, "max must be (N_dst, H)");
  DGLMI_CHECK(sm->shape[0] == in.num_rows && feat_numel(sm) == H, "sum must be (N_dst, H)");
  DGLMI_CHECK(aligned16(ft->data) && aligned16(out->data), "feat_src/out must be 16-byte aligned");
  GatArgs a;
  std::memset(&a, 0, sizeof(a));
  a.indptr = in.indptr;
  a.rows = in.rows;
  a.indices = in.indices;
  a.nnz = in.nnz;
  a.num_rows = in.num_rows;
  a.H = static_cast<int>(H);
  a.D = static_cast<int>(D);
  a.F = H * D;
  a.slope = slope;
  a.ft = ft->data;
  a.el = el->data;
  a.er = er->data;
  a.out = out->data;
  a.m = mx->data;
  a.l = sm->data;
  a.chunk = gat_chunk_edges(std::max<int64_t>(in.nnz, 1));
  a.o32 = std::max(ft->shape[0], in.num_rows) * a.F < (int64_t(1) << 31);
  return a;
}

}  // namespace

namespace dglmi {
void set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }
}  // namespace dglmi

extern "C" {

const char* DGLMIGetLastError(void) { return g_last_error.c_str(); }

const char* DGLMIVersion(void) { return "0.4-mi355x"; }

int DGLMISetSddmmOrder(int32_t order) {
  API_BEGIN();
  if (order != DGLMI_SDDMM_ORDER_AUTO && order != DGLMI_SDDMM_ORDER_COO &&
      order != DGLMI_SDDMM_ORDER_CSR)
    throw std::invalid_argument("DGLMISetSddmmOrder: order must be 0 (auto), 1 (coo) or 2 (csr)");
  g_sddmm_order.store(order, std::memory_order_relaxed);
  API_END();
}

int DGLMIKernelInferBinaryFeatureShape(const char* op, const DGLMIArray* lhs,
                                       const DGLMIArray* rhs, int64_t* out_shape,
                                       int32_t* out_ndim) {
  API_BEGIN();
  DGLMI_CHECK(lhs && rhs && out_shape && out_ndim, "null argument");
  std::vector<int64_t> ro;
  calc_bcast(parse_op(op), lhs, rhs, &ro);
  *out_ndim = static_cast<int32_t>(ro.size());
  for (size_t i = 0; i < ro.size(); ++i) out_shape[i] = ro[i];
  API_END();
}

int DGLMIKernelBinaryOpReduce(const char* reducer, const char* op, const DGLMIGraph* graph,
                              int32_t lhs_target, int32_t rhs_target, const DGLMIArray* lhs,
                              const DGLMIArray* rhs, DGLMIArray* out,
                              const int32_t* lhs_mapping, const int32_t* rhs_mapping,
                              const int32_t* out_mapping, void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  const int o = parse_op(op);
  check_graph(graph);
  check_maps(graph, lhs_mapping, rhs_mapping, out_mapping);
  DeviceGuard guard(graph->device);
  forward(red, o, graph, lhs_target, rhs_target, lhs, rhs, out, lhs_mapping, rhs_mapping,
          out_mapping, static_cast<hipStream_t>(stream));
  API_END();
}

int DGLMIKernelBinaryOpReduceEx(const char* reducer, const char* op, const DGLMIGraph* graph,
                                int32_t lhs_target, int32_t rhs_target, const DGLMIArray* lhs,
                                const DGLMIArray* rhs, DGLMIArray* out,
                                const int32_t* lhs_mapping, const int32_t* rhs_mapping,
                                const int32_t* out_mapping, const DGLMIEpilogue* epilogue,
                                void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  const int o = parse_op(op);
  check_graph(graph);
  check_maps(graph, lhs_mapping, rhs_mapping, out_mapping);
  DeviceGuard guard(graph->device);
  forward(red, o, graph, lhs_target, rhs_target, lhs, rhs, out, lhs_mapping, rhs_mapping,
          out_mapping, static_cast<hipStream_t>(stream), epilogue);
  API_END();
}

int DGLMIKernelBackwardLhsBinaryOpReduce(
    const char* reducer, const char* op, const DGLMIGraph* graph, int32_t lhs_target,
    int32_t rhs_target, const int32_t* lhs_mapping, const int32_t* rhs_mapping,
    const int32_t* out_mapping, const DGLMIArray* lhs, const DGLMIArray* rhs,
    const DGLMIArray* out, const DGLMIArray* grad_out, DGLMIArray* grad_lhs, void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  const int o = parse_op(op);
  check_graph(graph);
  check_maps(graph, lhs_mapping, rhs_mapping, out_mapping);
  DeviceGuard guard(graph->device);
  backward(red, o, graph, lhs_target, rhs_target, lhs_mapping, rhs_mapping, out_mapping, lhs, rhs,
           out, grad_out, grad_lhs, 0, static_cast<hipStream_t>(stream));
  API_END();
}

int DGLMIKernelBackwardRhsBinaryOpReduce(
    const char* reducer, const char* op, const DGLMIGraph* graph, int32_t lhs_target,
    int32_t rhs_target, const int32_t* lhs_mapping, const int32_t* rhs_mapping,
    const int32_t* out_mapping, const DGLMIArray* lhs, const DGLMIArray* rhs,
    const DGLMIArray* out, const DGLMIArray* grad_out, DGLMIArray* grad_rhs, void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  const int o = parse_op(op);
  check_graph(graph);
  check_maps(graph, lhs_mapping, rhs_mapping, out_mapping);
  DeviceGuard guard(graph->device);
  backward(red, o, graph, lhs_target, rhs_target, lhs_mapping, rhs_mapping, out_mapping, lhs, rhs,
           out, grad_out, grad_rhs, 1, static_cast<hipStream_t>(stream));
  API_END();
}

int DGLMIKernelCopyReduce(const char* reducer, const DGLMIGraph* graph, int32_t target,
                          const DGLMIArray* in, DGLMIArray* out, const int32_t* in_mapping,
                          const int32_t* out_mapping, void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  check_graph(graph);
  check_maps(graph, in_mapping, out_mapping, nullptr);
  DeviceGuard guard(graph->device);
  forward(red, OP_USE_LHS, graph, target, DGLMI_TARGET_NONE, in, nullptr, out, in_mapping,
          nullptr, out_mapping, static_cast<hipStream_t>(stream));
  API_END();
}

int DGLMIKernelCopyReduceEx(const char* reducer, const DGLMIGraph* graph, int32_t target,
                            const DGLMIArray* in, DGLMIArray* out, const int32_t* in_mapping,
                            const int32_t* out_mapping, const DGLMIEpilogue* epilogue,
                            void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  check_graph(graph);
  check_maps(graph, in_mapping, out_mapping, nullptr);
  DeviceGuard guard(graph->device);
  forward(red, OP_USE_LHS, graph, target, DGLMI_TARGET_NONE, in, nullptr, out, in_mapping,
          nullptr, out_mapping, static_cast<hipStream_t>(stream), epilogue);
  API_END();
}

int DGLMIKernelBackwardCopyReduce(const char* reducer, const DGLMIGraph* graph, int32_t target,
                                  const DGLMIArray* in, const DGLMIArray* out,
                                  const DGLMIArray* grad_out, DGLMIArray* grad_in,
                                  const int32_t* in_mapping, const int32_t* out_mapping,
                                  void* stream) {
  API_BEGIN();
  const int red = parse_reducer(reducer);
  check_graph(graph);
  check_maps(graph, in_mapping, out_mapping, nullptr);
  DeviceGuard guard(graph->device);
  backward(red, OP_USE_LHS, graph, target, DGLMI_TARGET_NONE, in_mapping, nullptr, out_mapping, in,
           nullptr, out, grad_out, grad_in, 0, static_cast<hipStream_t>(stream));
  API_END();
}

int DGLMIFusedGatSupported(int64_t heads, int64_t head_dim) {
  return gat_supported(heads, head_dim) ? 1 : 0;
}

}  // extern "C"

namespace {
// the optional slope aggregates of DGLMIFusedGatForwardEx / BackwardEx
void gat_check_ls(const GatArgs& a, const DGLMIArray* lf, const DGLMIArray* ls) {
  DGLMI_CHECK((lf == nullptr) == (ls == nullptr), "slope_feat and slope_sum go together");
  if (lf == nullptr) return;
  check_array(lf, "slope_feat");
  check_array(ls, "slope_sum");
  DGLMI_CHECK(lf->shape[0] == a.num_rows && feat_numel(lf) == a.F, "slope_feat must be (N_dst, H, D)");
  DGLMI_CHECK(ls->shape[0] == a.num_rows && feat_numel(ls) == a.H, "slope_sum must be (N_dst, H)");
  DGLMI_CHECK(aligned16(lf->data), "slope_feat must be 16-byte aligned");
}

// attention dropout parameters of the GatArgs (p = 0 and no keep words: off).  Hashed
// mask: 16-bit uniforms per edge and head (internal.h gat_head_keep), p resolved to
// 2^-16 as t = round(p 2^16); a weight is kept when its uniform is >= t, so the keep
// probability is (2^16 - t) / 2^16 and the scale its inverse (the rescaled expectation
// stays unbiased); t = 2^16 (p >= 1 - 2^-17, p = 1 included) keeps nothing, scale 0.
// Caller's mask (`keep`, one uint32 word per edge id, bit h = head h kept): the kernels
// read it through the walk's edge ids and scale kept weights by `keep_scale`.
// torch's own draws (`draw`, DGLMIFusedGatDraw*): the kernels recompute the fused dropout
// kernel's Philox draw of element e * H + h (internal.h dropout_draw_slot) for edge e.
void gat_set_draw(GatArgs& a, const DGLMIDropoutDraw* d, int64_t num_edges) {
  DGLMI_CHECK(d->vec == 1 || d->vec == 2 || d->vec == 4, "dropout draw: vec must be 1, 2 or 4");
  DGLMI_CHECK(d->threads >= 1, "dropout draw: threads >= 1");
  DGLMI_CHECK(d->offset % 4 == 0, "dropout draw: the generator offset is a multiple of 4");
  DGLMI_CHECK((num_edges * a.H) % d->vec == 0, "dropout draw: E x H is not a multiple of vec");
  DGLMI_CHECK(std::isfinite(d->keep) && d->keep >= 0.0f && d->keep <= 1.0f, "dropout draw: keep in [0, 1]");
  DGLMI_CHECK(std::isfinite(d->scale) && d->scale >= 0.0f, "dropout draw: scale finite and >= 0");
  a.drop = 1;
  a.drop_rng = 1;
  a.rng_seed = d->seed;
  a.rng_ctr = d->offset / 4;
  a.rng_threads = d->threads;
  a.rng_vec = d->vec;
  a.rng_shift = (d->threads & (d->threads - 1)) == 0 ? __builtin_ctzll(static_cast<uint64_t>(d->threads)) : -1;
  a.rng_keep = d->keep;
  a.drop_scale = d->scale;
}

void gat_set_dropout(GatArgs& a, float p, uint64_t seed, const void* keep = nullptr, int keep_bits = 0,
                     float keep_scale = 0.0f, int64_t num_edges = 0, int keep_pos = 0,
                     const DGLMIDropoutDraw* draw = nullptr) {
  if (draw != nullptr) {
    gat_set_draw(a, draw, num_edges);
  } else if (keep != nullptr || keep_bits != 0) {
    a.drop_pos = keep_pos != 0 ? 1 : 0;
    a.drop_off = 0;
    DGLMI_CHECK(keep_bits == 8 || keep_bits == 16 || keep_bits == 32, "keep_bits must be 8, 16 or 32");
    DGLMI_CHECK(a.H <= keep_bits, "keep words narrower than the head count");
    DGLMI_CHECK(keep != nullptr || num_edges == 0, "keep (one word per edge) is required");
    DGLMI_CHECK(std::isfinite(keep_scale) && keep_scale >= 0.0f, "keep_scale must be finite and >= 0");
    a.drop = 2;
    a.drop_bits = keep;
    a.drop_width = keep_bits;
    a.drop_scale = keep_scale;
  } else {
    DGLMI_CHECK(p >= 0.0f && p <= 1.0f, "attn_drop must be in [0, 1]");
    a.drop = p > 0.0f ? 1 : 0;
    if (!a.drop) return;
    const double t = std::min(65536.0, std::floor(static_cast<double>(p) * 65536.0 + 0.5));
    a.drop_thresh = static_cast<uint32_t>(t);
    a.drop_scale = t < 65536.0 ? static_cast<float>(65536.0 / (65536.0 - t)) : 0.0f;
    a.drop_seed = seed;
  }
  DGLMI_CHECK(a.o32, "attention dropout needs gathered tables below 2^31 elements");
  DGLMI_CHECK(a.H <= 32, "attention dropout in the fused kernels takes at most 32 heads");
}

int gat_forward_impl(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                     const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                     DGLMIArray* max_out, DGLMIArray* sum_out, DGLMIArray* lf, DGLMIArray* ls,
                     void* stream, float attn_drop = 0.0f, uint64_t seed = 0,
                     const void* keep = nullptr, int keep_bits = 0, float keep_scale = 0.0f,
                     int keep_pos = 0, const DGLMIDropoutDraw* draw = nullptr) {
  API_BEGIN();
  check_graph32(graph, "fused GAT");
  DeviceGuard guard(graph->device);
  GatArgs a = gat_args(graph, feat_src, el, er, negative_slope, out, max_out, sum_out);
  gat_check_ls(a, lf, ls);
  gat_set_dropout(a, attn_drop, seed, keep, keep_bits, keep_scale, graph->in_csr.nnz, keep_pos, draw);
  a.eids = graph->in_csr.data;
  a.lf = lf ? lf->data : nullptr;
  a.ls = ls ? ls->data : nullptr;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const DGLMICsr& walk = graph->in_csr;
  if (a.num_rows * a.F == 0) return 0;
  if (walk.nnz == 0) {
    launch_fill(out->data, a.num_rows * a.F, 0.0f, s);
    launch_fill(max_out->data, a.num_rows * a.H, 0.0f, s);
    launch_fill(sum_out->data, a.num_rows * a.H, 0.0f, s);
    if (lf) {
      launch_fill(lf->data, a.num_rows * a.F, 0.0f, s);
      launch_fill(ls->data, a.num_rows * a.H, 0.0f, s);
    }
    return 0;
  }
  // carry record per chunk: acc, m, l (+ lf, ls)
  const int64_t cw = lf ? 2 * a.F + 3 * a.H : a.F + 2 * a.H;
  const int nb = gat_blocks(graph);
  if (nb > 1) {
    // column-blocked: one raw (unnormalised) launch per source block into its own
    // partial buffers, then the in-order merge
    const int64_t N = a.num_rows;
    const int64_t part_floats = nb * N * cw;
    int64_t max_chunks = 0;
    for (int b = 0; b < nb; ++b) {
      const int64_t c = graph->in_col_blocks[b].nnz;
      max_chunks = std::max(max_chunks, (c + gat_chunk_edges(std::max<int64_t>(c, 1)) - 1) /
                                            gat_chunk_edges(std::max<int64_t>(c, 1)));
    }
    const int64_t part_bytes = (part_floats * static_cast<int64_t>(sizeof(float)) + 255) & ~int64_t(255);
    const int64_t carry_bytes = (max_chunks * cw * static_cast<int64_t>(sizeof(float)) + 15) & ~int64_t(15);
    Scratch ws(graph, part_bytes + carry_bytes + max_chunks * static_cast<int64_t>(sizeof(int32_t)), s);
    // [out parts][lf parts][m parts][l parts][ls parts]: the float4 arrays first
    float* out_part = static_cast<float*>(ws.ptr);
    float* lf_part = lf ? out_part + nb * N * a.F : nullptr;
    float* m_part = out_part + nb * N * a.F * (lf ? 2 : 1);
    float* l_part = m_part + nb * N * a.H;
    float* ls_part = lf ? l_part + nb * N * a.H : nullptr;
    int64_t keep_off = 0;  // position-ordered keep words: the blocks in order
    for (int b = 0; b < nb; ++b) {
      const DGLMICsr& c = graph->in_col_blocks[b];
      GatArgs ab = a;
      ab.drop_off = keep_off;
      keep_off += c.nnz;
      ab.indptr = c.indptr;
      ab.rows = c.rows;
      ab.indices = c.indices;
      ab.eids = c.data;
      ab.nnz = c.nnz;
      ab.chunk = gat_chunk_edges(std::max<int64_t>(c.nnz, 1));
      ab.out = out_part + b * N * a.F;
      ab.m = m_part + b * N * a.H;
      ab.l = l_part + b * N * a.H;
      if (lf) {
        ab.lf = lf_part + b * N * a.F;
        ab.ls = ls_part + b * N * a.H;
      }
      ab.raw = 1;
      ab.carry = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + part_bytes);
      ab.seg_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(ws.ptr) + part_bytes + carry_bytes);
      launch_gat_forward(ab, s);
    }
    launch_gat_merge(out_part, m_part, l_part, nb, N, a.H, a.D, out->data, max_out->data,
                     sum_out->data, s, lf_part, ls_part, lf ? lf->data : nullptr,
                     ls ? ls->data : nullptr);
    check_hip(hipGetLastError(), "fused GAT forward (blocked) launch");
    return 0;
  }
  const int64_t chunks = (walk.nnz + a.chunk - 1) / a.chunk;
  const int64_t carry_bytes = (chunks * cw * static_cast<int64_t>(sizeof(float)) + 15) & ~int64_t(15);
  Scratch carry(graph, carry_bytes + chunks * static_cast<int64_t>(sizeof(int32_t)), s);
  a.carry = static_cast<float*>(carry.ptr);
  a.seg_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(carry.ptr) + carry_bytes);
  launch_gat_forward(a, s);
  check_hip(hipGetLastError(), "fused GAT forward launch");
  API_END();
}
}  // namespace

extern "C" {

int DGLMIFusedGatForward(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                         const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                         DGLMIArray* max_out, DGLMIArray* sum_out, void* stream) {
  return gat_forward_impl(graph, feat_src, el, er, negative_slope, out, max_out, sum_out, nullptr,
                          nullptr, stream);
}

int DGLMIFusedGatForwardEx(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                           const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                           DGLMIArray* max_out, DGLMIArray* sum_out, DGLMIArray* slope_feat,
                           DGLMIArray* slope_sum, void* stream) {
  return gat_forward_impl(graph, feat_src, el, er, negative_slope, out, max_out, sum_out, slope_feat,
                          slope_sum, stream);
}

}  // extern "C"

namespace {
int gat_backward_impl(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                      const DGLMIArray* er, float negative_slope, const DGLMIArray* out,
                      const DGLMIArray* max_in, const DGLMIArray* sum_in, const DGLMIArray* lf_in,
                      const DGLMIArray* ls_in, const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                      DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream, float attn_drop = 0.0f,
                      uint64_t seed = 0, const void* keep = nullptr, int keep_bits = 0,
                      float keep_scale = 0.0f, int keep_pos = 0, const DGLMIDropoutDraw* draw = nullptr) {
  API_BEGIN();
  check_graph32(graph, "fused GAT");
  DeviceGuard guard(graph->device);
  GatArgs a = gat_args(graph, feat_src, el, er, negative_slope, const_cast<DGLMIArray*>(out),
                       const_cast<DGLMIArray*>(max_in), const_cast<DGLMIArray*>(sum_in));
  gat_set_dropout(a, attn_drop, seed, keep, keep_bits, keep_scale, graph->in_csr.nnz, keep_pos, draw);
  // with dropout only the slope-aggregate backward (no destination-side walk) applies
  // with dropout only the slope-aggregate backward applies -- or, for the recomputed
  // draws (drop_rng), the destination-side walks too (GATConv's composition keeps no
  // slope aggregates); never the edge-position path
  DGLMI_CHECK(!a.drop || lf_in != nullptr || a.drop_rng,
              "attention dropout needs the forward's slope aggregates (slope_feat / slope_sum)");
  hipStream_t s = static_cast<hipStream_t>(stream);
  a.chunk = gat_bwd_chunk_edges(std::max<int64_t>(graph->in_csr.nnz, 1));
  check_array(grad_out, "grad_out");
  check_array(grad_feat_src, "grad_feat_src");
  check_array(grad_el, "grad_el");
  check_array(grad_er, "grad_er");
  const int64_t n_src = feat_src->shape[0];
  DGLMI_CHECK(grad_out->shape[0] == a.num_rows && feat_numel(grad_out) == a.F, "grad_out shape");
  DGLMI_CHECK(grad_feat_src->shape[0] == n_src && feat_numel(grad_feat_src) == a.F, "grad_feat_src shape");
  DGLMI_CHECK(grad_el->shape[0] == n_src && feat_numel(grad_el) == a.H, "grad_el shape");
  DGLMI_CHECK(grad_er->shape[0] == a.num_rows && feat_numel(grad_er) == a.H, "grad_er shape");
  const DGLMICsr& in = graph->in_csr;
  const DGLMICsr& outc = graph->out_csr;
  check_csr(outc, "out_csr", true);
  DGLMI_CHECK(outc.num_rows == n_src, "out_csr rows != feat_src rows");
  if (in.nnz == 0) {
    launch_fill(grad_feat_src->data, n_src * a.F, 0.0f, s);
    launch_fill(grad_el->data, n_src * a.H, 0.0f, s);
    launch_fill(grad_er->data, a.num_rows * a.H, 0.0f, s);
    return 0;
  }
  a.go = grad_out->data;
  a.fo = out->data;
  a.m_in = max_in->data;
  a.l_in = sum_in->data;
  a.g_er = grad_er->data;
  a.g_el = grad_el->data;
  a.g_ft = grad_feat_src->data;
  gat_check_ls(a, lf_in, ls_in);
  const int nb = gat_blocks(graph);
  // Edge-position backward (DGLMIGraph.gat_edge_pos): no destination-side walk.  The
  // stats come from a dense pass, the source-side walk stores every edge's grad_er
  // term in out-CSR order, and grad_er is one copy_e-style gather-sum over the in-CSR
  // through the position map -- a 32-B term per edge instead of a 256-B feature row
  // and a logit (C3 unblocked, H = 8: backward 11.98 -> 9.57 ms; M1-size RMAT
  // 11.48 -> 10.89 ms).  Unblocked walks only: with column blocks the destination
  // walk's gathers hit L2 and the term writes plus their random re-reads cost more
  // (C3, 8 blocks: 8.52 -> 9.15 ms; profiles/r03_gat_edge_pos.json).
  const bool blocks_given = graph->num_col_blocks > 1 && graph->in_col_blocks != nullptr &&
                            graph->out_col_blocks != nullptr;
  const bool pos_path = !a.drop && graph->gat_edge_pos != nullptr && nb == 1 && !blocks_given &&
                        fast_supported(FAST_COPY_EDGE, a.H, 1) && aligned16(grad_er->data);
  int64_t chunks = (in.nnz + a.chunk - 1) / a.chunk;
  for (int b = 0; b < nb && nb > 1; ++b)
    for (const DGLMICsr* c : {&graph->in_col_blocks[b], &graph->out_col_blocks[b]}) {
      const int64_t k = gat_bwd_chunk_edges(std::max<int64_t>(c->nnz, 1));
      chunks = std::max(chunks, (c->nnz + k - 1) / k);
    }
  const int64_t stats_bytes = a.num_rows * a.H * 16;
  const int64_t carry_bytes = (chunks * (a.F + a.H) * static_cast<int64_t>(sizeof(float)) + 15) & ~int64_t(15);
  Scratch ws(graph, stats_bytes + carry_bytes + chunks * static_cast<int64_t>(sizeof(int32_t)) + 256, s);
  a.stats = static_cast<float4*>(ws.ptr);
  a.carry = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + ((stats_bytes + 255) & ~int64_t(255)));
  a.seg_cnt = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(a.carry) + carry_bytes);
  if (lf_in != nullptr) {
    // the forward kept the slope aggregates: stats and grad_er from one dense pass, then
    // the source-side walk(s) only -- no destination-side walk, no per-edge terms
    a.lf = lf_in->data;
    a.ls = ls_in->data;
    launch_gat_stats(a, s);
    a.lf = a.ls = nullptr;
    int64_t keep_off = 0;  // position-ordered keep words: the out-blocks in order
    auto src_walk = [&](const DGLMICsr& c, bool accumulate) {
      GatArgs b = a;
      b.drop_off = keep_off;
      keep_off += c.nnz;
      b.indptr = c.indptr;
      b.rows = c.rows;
      b.indices = c.indices;
      b.eids = c.data;
      b.nnz = c.nnz;
      b.num_rows = c.num_rows;
      b.chunk = gat_bwd_chunk_edges(std::max<int64_t>(c.nnz, 1));
      b.accumulate = accumulate;
      launch_gat_backward_src(b, s);
    };
    if (nb > 1)
      for (int b = 0; b < nb; ++b) src_walk(graph->out_col_blocks[b], b > 0);
    else
      src_walk(outc, false);
    check_hip(hipGetLastError(), "fused GAT backward (slope aggregates) launch");
    return 0;
  }
  if (pos_path) {
    DGLMIGraph nows;  // t must not alias the caller's workspace (the reduce's carries)
    std::memset(&nows, 0, sizeof(nows));
    Scratch tbuf(&nows, in.nnz * a.H * static_cast<int64_t>(sizeof(float)), s);
    a.t = static_cast<float*>(tbuf.ptr);
    launch_gat_stats(a, s);
    GatArgs b = a;
    b.indptr = outc.indptr;
    b.rows = outc.rows;
    b.indices = outc.indices;
    b.nnz = outc.nnz;
    b.num_rows = outc.num_rows;
    launch_gat_backward_src(b, s);
    check_hip(hipGetLastError(), "fused GAT backward (src) launch");
    DGLMIGraph gp = *graph;  // no blocks / hints for the gather-sum
    gp.num_col_blocks = 0;
    gp.in_col_blocks = gp.out_col_blocks = nullptr;
    gp.in_gather_cols = gp.out_gather_cols = nullptr;
    DGLMICsr walk = in;
    walk.data = graph->gat_edge_pos;
    run_fast(&gp, walk, FAST_COPY_EDGE, RED_SUM, a.t, nullptr, nullptr, nullptr, grad_er->data, a.H,
             1, s);
    return 0;
  }
  if (nb > 1) {
    // column-blocked: block 0 writes every row's stats and the first gradient
    // terms, later blocks add theirs (block order), first the destination side
    // over the source blocks, then the source side over the destination blocks
    auto set_walk = [](GatArgs& g, const DGLMICsr& c) {
      g.indptr = c.indptr;
      g.rows = c.rows;
      g.indices = c.indices;
      g.eids = c.data;
      g.nnz = c.nnz;
      g.num_rows = c.num_rows;
      g.chunk = gat_bwd_chunk_edges(std::max<int64_t>(c.nnz, 1));
    };
    for (int b = 0; b < nb; ++b) {
      GatArgs ab = a;
      set_walk(ab, graph->in_col_blocks[b]);
      ab.accumulate = b > 0;
      ab.skip_stats = b > 0;
      launch_gat_backward_dst(ab, s);
    }
    for (int b = 0; b < nb; ++b) {
      GatArgs ab = a;
      set_walk(ab, graph->out_col_blocks[b]);
      ab.accumulate = b > 0;
      launch_gat_backward_src(ab, s);
    }
    check_hip(hipGetLastError(), "fused GAT backward (blocked) launch");
    return 0;
  }
  // destination side on the in-CSR
  a.eids = in.data;
  launch_gat_backward_dst(a, s);
  check_hip(hipGetLastError(), "fused GAT backward (dst) launch");
  // source side on the out-CSR
  GatArgs b = a;
  b.indptr = outc.indptr;
  b.rows = outc.rows;
  b.indices = outc.indices;
  b.eids = outc.data;
  b.nnz = outc.nnz;
  b.num_rows = outc.num_rows;
  launch_gat_backward_src(b, s);
  check_hip(hipGetLastError(), "fused GAT backward (src) launch");
  API_END();
}

}  // namespace

extern "C" {

int DGLMIFusedGatBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                          const DGLMIArray* er, float negative_slope, const DGLMIArray* out,
                          const DGLMIArray* max_in, const DGLMIArray* sum_in,
                          const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                          DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream) {
  return gat_backward_impl(graph, feat_src, el, er, negative_slope, out, max_in, sum_in, nullptr,
                           nullptr, grad_out, grad_feat_src, grad_el, grad_er, stream);
}

int DGLMIFusedGatBackwardEx(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                            const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                            const DGLMIArray* out, const DGLMIArray* max_in,
                            const DGLMIArray* sum_in, const DGLMIArray* slope_feat,
                            const DGLMIArray* slope_sum, const DGLMIArray* grad_out,
                            DGLMIArray* grad_feat_src, DGLMIArray* grad_el, DGLMIArray* grad_er,
                            void* stream) {
  return gat_backward_impl(graph, feat_src, el, er, negative_slope, out, max_in, sum_in, slope_feat,
                           slope_sum, grad_out, grad_feat_src, grad_el, grad_er, stream);
}

int DGLMIFusedGatDropoutForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                                float attn_drop, uint64_t seed, DGLMIArray* out, DGLMIArray* max_out,
                                DGLMIArray* sum_out, DGLMIArray* slope_feat, DGLMIArray* slope_sum,
                                void* stream) {
  return gat_forward_impl(graph, feat_src, el, er, negative_slope, out, max_out, sum_out, slope_feat,
                          slope_sum, stream, attn_drop, seed);
}

int DGLMIFusedGatDropoutBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                 const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                                 float attn_drop, uint64_t seed, const DGLMIArray* out,
                                 const DGLMIArray* max_in, const DGLMIArray* sum_in,
                                 const DGLMIArray* slope_feat, const DGLMIArray* slope_sum,
                                 const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                                 DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream) {
  return gat_backward_impl(graph, feat_src, el, er, negative_slope, out, max_in, sum_in, slope_feat,
                           slope_sum, grad_out, grad_feat_src, grad_el, grad_er, stream, attn_drop,
                           seed);
}

int DGLMIFusedGatKeepForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                             const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                             const void* keep, int keep_bits, int keep_by_position, float keep_scale,
                             DGLMIArray* out, DGLMIArray* max_out, DGLMIArray* sum_out,
                             DGLMIArray* slope_feat, DGLMIArray* slope_sum, void* stream) {
  if (keep_bits == 0) {
    g_last_error = "keep_bits must be 8, 16 or 32";
    return -1;
  }
  return gat_forward_impl(graph, feat_src, el, er, negative_slope, out, max_out, sum_out, slope_feat,
                          slope_sum, stream, 0.0f, 0, keep, keep_bits, keep_scale, keep_by_position);
}

int DGLMIFusedGatKeepBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                              const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                              const void* keep, int keep_bits, int keep_by_position, float keep_scale,
                              const DGLMIArray* out, const DGLMIArray* max_in, const DGLMIArray* sum_in,
                              const DGLMIArray* slope_feat, const DGLMIArray* slope_sum,
                              const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                              DGLMIArray* grad_el, DGLMIArray* grad_er, void* stream) {
  if (keep_bits == 0) {
    g_last_error = "keep_bits must be 8, 16 or 32";
    return -1;
  }
  return gat_backward_impl(graph, feat_src, el, er, negative_slope, out, max_in, sum_in, slope_feat,
                           slope_sum, grad_out, grad_feat_src, grad_el, grad_er, stream, 0.0f, 0,
                           keep, keep_bits, keep_scale, keep_by_position);
}

int DGLMIFusedGatDrawForward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                             const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                             const DGLMIDropoutDraw* draw, DGLMIArray* out, DGLMIArray* max_out,
                             DGLMIArray* sum_out, DGLMIArray* slope_feat, DGLMIArray* slope_sum, void* stream) {
  if (draw == nullptr) {
    g_last_error = "DGLMIFusedGatDrawForward: draw is required";
    return -1;
  }
  return gat_forward_impl(graph, feat_src, el, er, negative_slope, out, max_out, sum_out, slope_feat,
                          slope_sum, stream, 0.0f, 0, nullptr, 0, 0.0f, 0, draw);
}

int DGLMIFusedGatDrawBackward(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                              const DGLMIArray* el, const DGLMIArray* er, float negative_slope,
                              const DGLMIDropoutDraw* draw, const DGLMIArray* out, const DGLMIArray* max_in,
                              const DGLMIArray* sum_in, const DGLMIArray* slope_feat,
                              const DGLMIArray* slope_sum, const DGLMIArray* grad_out,
                              DGLMIArray* grad_feat_src, DGLMIArray* grad_el, DGLMIArray* grad_er,
                              void* stream) {
  if (draw == nullptr) {
    g_last_error = "DGLMIFusedGatDrawBackward: draw is required";
    return -1;
  }
  return gat_backward_impl(graph, feat_src, el, er, negative_slope, out, max_in, sum_in, slope_feat,
                           slope_sum, grad_out, grad_feat_src, grad_el, grad_er, stream, 0.0f, 0,
                           nullptr, 0, 0.0f, 0, draw);
}

int DGLMIDropoutDrawMask(const DGLMIDropoutDraw* draw, int64_t n, uint8_t* mask, void* stream) {
  API_BEGIN();
  DGLMI_CHECK(draw != nullptr, "DGLMIDropoutDrawMask: draw is required");
  DGLMI_CHECK(n >= 0 && (n == 0 || mask != nullptr), "DGLMIDropoutDrawMask: n >= 0, mask");
  DGLMI_CHECK(draw->vec == 1 || draw->vec == 2 || draw->vec == 4, "DGLMIDropoutDrawMask: vec 1, 2 or 4");
  DGLMI_CHECK(draw->threads >= 1 && draw->offset % 4 == 0, "DGLMIDropoutDrawMask: threads >= 1, offset % 4 == 0");
  DGLMI_CHECK(n % draw->vec == 0, "DGLMIDropoutDrawMask: n is not a multiple of vec");
  const int shift =
      (draw->threads & (draw->threads - 1)) == 0 ? __builtin_ctzll(static_cast<uint64_t>(draw->threads)) : -1;
  launch_dropout_draw_mask(draw->seed, draw->offset / 4, draw->threads, draw->vec, shift, draw->keep, n, mask,
                           static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "dropout draw mask launch");
  API_END();
}

namespace {
int dropout_draw_scale_impl(const DGLMIDropoutDraw* draw, int heads, const int32_t* eids, int64_t n, float* out,
                            bool apply, void* stream) {
  API_BEGIN();
  DGLMI_CHECK(draw != nullptr, "DGLMIDropoutDrawScale: draw is required");
  DGLMI_CHECK(heads >= 1 && heads <= 32, "DGLMIDropoutDrawScale: 1 <= heads <= 32");
  DGLMI_CHECK(n >= 0 && (n == 0 || out != nullptr), "DGLMIDropoutDrawScale: n >= 0, out");
  DGLMI_CHECK(n < (int64_t(1) << 31), "DGLMIDropoutDrawScale: positions below 2^31 (32-bit edge ids)");
  GatArgs a;
  std::memset(&a, 0, sizeof(a));
  a.H = heads;
  gat_set_draw(a, draw, n);
  launch_dropout_draw_scale(a, eids, n, out, apply, static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "dropout draw scale launch");
  API_END();
}
}  // namespace

int DGLMIDropoutDrawScale(const DGLMIDropoutDraw* draw, int heads, const int32_t* eids, int64_t n, float* out,
                          void* stream) {
  return dropout_draw_scale_impl(draw, heads, eids, n, out, false, stream);
}

int DGLMIDropoutDrawApply(const DGLMIDropoutDraw* draw, int heads, const int32_t* eids, int64_t n, float* x,
                          void* stream) {
  return dropout_draw_scale_impl(draw, heads, eids, n, x, true, stream);
}

int DGLMIGatKeepGather(const void* keep, int keep_bits, const int32_t* index, int64_t n, void* out,
                       void* stream) {
  API_BEGIN();
  DGLMI_CHECK(keep_bits == 8 || keep_bits == 16 || keep_bits == 32, "DGLMIGatKeepGather: keep_bits 8, 16 or 32");
  DGLMI_CHECK(n >= 0, "DGLMIGatKeepGather: n >= 0");
  DGLMI_CHECK(n == 0 || (keep != nullptr && index != nullptr && out != nullptr), "DGLMIGatKeepGather: null operand");
  launch_gat_keep_gather(keep, keep_bits, index, n, out, static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "keep gather launch");
  API_END();
}

int DGLMIGatKeepBits(const float* table, int64_t num_edges, int heads, void* bits, int keep_bits,
                     void* stream) {
  API_BEGIN();
  DGLMI_CHECK(keep_bits == 8 || keep_bits == 16 || keep_bits == 32, "DGLMIGatKeepBits: keep_bits 8, 16 or 32");
  DGLMI_CHECK(num_edges >= 0 && heads >= 1 && heads <= keep_bits, "DGLMIGatKeepBits: 1 <= heads <= keep_bits");
  DGLMI_CHECK(num_edges == 0 || (table != nullptr && bits != nullptr), "DGLMIGatKeepBits: null operand");
  launch_gat_keep_bits(table, num_edges, heads, bits, keep_bits, static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "keep bits launch");
  API_END();
}

int DGLMIGatKeepBitsMask(const uint8_t* mask, int64_t num_edges, int heads, void* bits, int keep_bits,
                         void* stream) {
  API_BEGIN();
  DGLMI_CHECK(keep_bits == 8 || keep_bits == 16 || keep_bits == 32, "DGLMIGatKeepBitsMask: keep_bits 8, 16 or 32");
  DGLMI_CHECK(num_edges >= 0 && heads >= 1 && heads <= keep_bits, "DGLMIGatKeepBitsMask: 1 <= heads <= keep_bits");
  DGLMI_CHECK(num_edges == 0 || (mask != nullptr && bits != nullptr), "DGLMIGatKeepBitsMask: null operand");
  DGLMI_CHECK(heads != 8 || reinterpret_cast<uintptr_t>(mask) % 8 == 0,
              "DGLMIGatKeepBitsMask: an 8-head mask must be 8-byte aligned");
  launch_gat_keep_bits_mask(mask, num_edges, heads, bits, keep_bits, static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "keep bits (mask) launch");
  API_END();
}

// The reference's argument order (_CAPI_DGLFusedGatKernel /
// _CAPI_DGLKernelBackwardFusedGat, binary_reduce.cc:380-396, 529-549) over the
// kernels above.  The caller owns `sum` (N, H[, 1]) and `exp` (E, H[, 1]) and
// hands both from the forward to the backward untouched (tensor.py:383-420); what
// they hold is this library's softmax state, not the hack's per-edge exponentials:
// when exp has room for N_dst * H floats it keeps the running max and sum the
// sum of exp(s - max); otherwise sum keeps max + log(sum) and exp is unused.
namespace {
bool gat_exp_holds_max(const DGLMIGraph* g, const DGLMIArray* feat_src, const DGLMIArray* sum,
                       const DGLMIArray* exp) {
  check_array(sum, "sum");
  check_array(exp, "exp");
  DGLMI_CHECK(feat_src != nullptr && feat_src->ndim == 3, "feat_src must be (N, H, D)");
  const int64_t H = feat_src->shape[1];
  DGLMI_CHECK(exp->shape[0] == g->in_csr.nnz && feat_numel(exp) == H, "exp must be (E, H[, 1])");
  DGLMI_CHECK(sum->shape[0] == g->in_csr.num_rows && feat_numel(sum) == H, "sum must be (N_dst, H[, 1])");
  return g->in_csr.nnz >= g->in_csr.num_rows;
}
DGLMIArray gat_state_view(float* data, int64_t rows, int64_t H, int64_t D = 0) {
  DGLMIArray v;
  std::memset(&v, 0, sizeof(v));
  v.data = data;
  v.ndim = D > 0 ? 3 : 2;
  v.shape[0] = rows;
  v.shape[1] = H;
  v.shape[2] = D;
  return v;
}
// exp (E, H) also holds the slope aggregates after the running max: slope_feat
// (N, H, D) from float round_up(N H, 4), then slope_sum (N, H) -- room for all three
// when E >= N (D + 2) about (C3: E / N ~ 490); then the backward runs no
// destination-side walk (DGLMIFusedGatForwardEx)
int64_t gat_lf_offset(int64_t N, int64_t H) { return (N * H + 3) & ~int64_t(3); }
bool gat_exp_holds_slopes(const DGLMIGraph* g, const DGLMIArray* feat_src, const DGLMIArray* exp) {
  const int64_t N = g->in_csr.num_rows, E = g->in_csr.nnz;
  const int64_t H = feat_src->shape[1], D = feat_src->shape[2];
  return aligned16(exp->data) && E * H >= gat_lf_offset(N, H) + N * H * D + N * H;
}
}  // namespace

int DGLMIFusedGatKernel(const DGLMIGraph* graph, const DGLMIArray* feat_src, const DGLMIArray* el,
                        const DGLMIArray* er, DGLMIArray* sum, DGLMIArray* exp, DGLMIArray* ret,
                        float slope, void* stream) {
  API_BEGIN();
  check_graph32(graph, "fused GAT");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t N = graph->in_csr.num_rows, H = feat_src ? feat_src->shape[1] : 0;
  DGLMIArray l = gat_state_view(sum->data, N, H);
  if (gat_exp_holds_max(graph, feat_src, sum, exp)) {
    DGLMIArray m = gat_state_view(exp->data, N, H);
    if (gat_exp_holds_slopes(graph, feat_src, exp)) {
      const int64_t D = feat_src->shape[2];
      DGLMIArray lf = gat_state_view(exp->data + gat_lf_offset(N, H), N, H, D);
      DGLMIArray ls = gat_state_view(lf.data + N * H * D, N, H);
      if (DGLMIFusedGatForwardEx(graph, feat_src, el, er, slope, ret, &m, &l, &lf, &ls, stream) != 0)
        throw Error(g_last_error);
    } else if (DGLMIFusedGatForward(graph, feat_src, el, er, slope, ret, &m, &l, stream) != 0) {
      throw Error(g_last_error);
    }
  } else {
    DGLMIGraph no_ws = *graph;  // the max must not alias the kernels' workspace
    no_ws.workspace = nullptr;
    no_ws.workspace_bytes = 0;
    Scratch mx(&no_ws, N * H * static_cast<int64_t>(sizeof(float)), s);
    DGLMIArray m = gat_state_view(static_cast<float*>(mx.ptr), N, H);
    if (DGLMIFusedGatForward(graph, feat_src, el, er, slope, ret, &m, &l, stream) != 0)
      throw Error(g_last_error);
    launch_gat_fold_lse(m.data, l.data, N * H, s);
    check_hip(hipGetLastError(), "fused GAT log-sum-exp");
  }
  API_END();
}

int DGLMIKernelBackwardFusedGat(const DGLMIGraph* graph, const DGLMIArray* feat_src,
                                const DGLMIArray* el, const DGLMIArray* er, const DGLMIArray* sum,
                                const DGLMIArray* exp, const DGLMIArray* ret,
                                const DGLMIArray* grad_out, DGLMIArray* grad_feat_src,
                                DGLMIArray* grad_el, DGLMIArray* grad_er, float slope,
                                void* stream) {
  API_BEGIN();
  check_graph32(graph, "fused GAT");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t N = graph->in_csr.num_rows, H = feat_src ? feat_src->shape[1] : 0;
  if (gat_exp_holds_max(graph, feat_src, sum, exp)) {
    const DGLMIArray m = gat_state_view(exp->data, N, H);
    const DGLMIArray l = gat_state_view(sum->data, N, H);
    if (gat_exp_holds_slopes(graph, feat_src, exp)) {
      const int64_t D = feat_src->shape[2];
      const DGLMIArray lf = gat_state_view(exp->data + gat_lf_offset(N, H), N, H, D);
      const DGLMIArray ls = gat_state_view(lf.data + N * H * D, N, H);
      if (DGLMIFusedGatBackwardEx(graph, feat_src, el, er, slope, ret, &m, &l, &lf, &ls, grad_out,
                                  grad_feat_src, grad_el, grad_er, stream) != 0)
        throw Error(g_last_error);
    } else if (DGLMIFusedGatBackward(graph, feat_src, el, er, slope, ret, &m, &l, grad_out,
                                     grad_feat_src, grad_el, grad_er, stream) != 0) {
      throw Error(g_last_error);
    }
  } else {
    // sum holds max + log(sum): attention = exp(s - lse) / 1
    DGLMIGraph no_ws = *graph;
    no_ws.workspace = nullptr;
    no_ws.workspace_bytes = 0;
    Scratch ones(&no_ws, N * H * static_cast<int64_t>(sizeof(float)), s);
    launch_fill(static_cast<float*>(ones.ptr), N * H, 1.0f, s);
    const DGLMIArray m = gat_state_view(sum->data, N, H);
    const DGLMIArray l = gat_state_view(static_cast<float*>(ones.ptr), N, H);
    if (DGLMIFusedGatBackward(graph, feat_src, el, er, slope, ret, &m, &l, grad_out, grad_feat_src,
                              grad_el, grad_er, stream) != 0)
      throw Error(g_last_error);
  }
  API_END();
}

int DGLMIKernelMarkColdColumns(const DGLMIGraph* graph, int32_t direction,
                               int32_t min_hot_degree, int32_t* out_cols, void* stream) {
  API_BEGIN();
  check_graph(graph);
  DGLMI_CHECK(direction == 0 || direction == 1, "direction must be 0 (in-CSR) or 1 (out-CSR)");
  const DGLMICsr& c = direction == 0 ? graph->in_csr : graph->out_csr;
  const DGLMICsr& o = direction == 0 ? graph->out_csr : graph->in_csr;
  check_csr(c, direction == 0 ? "in_csr" : "out_csr", false, wide(graph));
  DGLMI_CHECK(o.indptr != nullptr && o.num_rows == c.num_cols,
              "the opposite CSR must have one row per column node");
  if (c.nnz > 0) DGLMI_CHECK(out_cols != nullptr, "null out_cols");
  DeviceGuard guard(graph->device);
  launch_mark_cold(c.indices, c.nnz, idx(graph, o.indptr), min_hot_degree, out_cols,
                   static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "mark cold columns launch");
  API_END();
}

int64_t DGLMIKernelWorkspaceBytes(const DGLMICsr* csr, int64_t feat_len) {
  if (csr == nullptr || csr->nnz <= 0 || feat_len <= 0) return 0;
  return fast_workspace_bytes(csr->nnz, feat_len);
}

int DGLMIEdgeSoftmaxSupported(int64_t values_per_edge) {
  return softmax_supported(values_per_edge) ? 1 : 0;
}

namespace {
// The edge softmax's workspace: the row statistics (max | sum, or S; unless the caller's),
// then the chunk carries and one segmented-fixup counter per chunk (the row-owned walk's
// carries fit in the same room), then the forward edge pass's packed row statistics
// (edge-id order: each row's max and sum side by side, one request per edge).
int64_t round256(int64_t b) { return (b + 255) & ~int64_t(255); }
int64_t softmax_carry_bytes(int64_t nnz, int64_t H) {
  const int64_t K = softmax_chunk_edges(nnz, H);
  const int64_t chunks = (nnz + K - 1) / K;
  const int64_t chunked = ((chunks * 2 * H * 4 + 15) & ~int64_t(15)) + chunks * 4;
  return round256(std::max(chunked, softmax_owned_carry_bytes(nnz, H)));
}
}  // namespace

int64_t DGLMIEdgeSoftmaxWorkspaceBytes(const DGLMICsr* in_csr, int64_t values_per_edge) {
  if (in_csr == nullptr || in_csr->nnz <= 0 || values_per_edge <= 0) return 0;
  const int64_t rows = in_csr->num_rows, H = values_per_edge;
  return round256(2 * rows * H * 4) + softmax_carry_bytes(in_csr->nnz, H) + round256(2 * rows * H * 4);
}

namespace {
// Points the softmax arguments into its workspace (DGLMIEdgeSoftmaxWorkspaceBytes's layout);
// own_stats: the row statistics live there too (else the caller set stat0 / stat1).
void softmax_layout(dglmi::SoftmaxArgs& a, void* ws, bool own_stats) {
  const int64_t H = a.H;
  char* base = static_cast<char*>(ws);
  if (own_stats) {
    a.stat0 = reinterpret_cast<float*>(base);
    a.stat1 = a.stat0 + a.num_rows * H;
  }
  a.carry = reinterpret_cast<float*>(base + round256(2 * a.num_rows * H * 4));
  a.seg_cnt = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(a.carry) +
                                         ((((a.nnz + a.chunk - 1) / a.chunk) * 2 * H * 4 + 15) & ~int64_t(15)));
  if (a.pack) a.stat_pk = reinterpret_cast<float*>(reinterpret_cast<char*>(a.carry) + softmax_carry_bytes(a.nnz, H));
}

// Shared checks of the edge-softmax entry points; returns H.
int64_t softmax_setup(const DGLMIGraph* g, const DGLMIArray* x, const char* name,
                      dglmi::SoftmaxArgs& a) {
  check_graph(g);
  check_array(x, name);
  const DGLMICsr& in = g->in_csr;
  check_csr(in, "in_csr", true, wide(g));
  DGLMI_CHECK(x->shape[0] >= in.nnz, std::string(name) + " has fewer rows than edges");
  const int64_t H = feat_numel(x);
  DGLMI_CHECK(softmax_supported(H), "edge softmax supports 1, 2, 4, 8 or 16 values per edge");
  DGLMI_CHECK(aligned16(x->data), std::string(name) + " must be 16-byte aligned");
  std::memset(&a, 0, sizeof(a));
  a.indptr = idx(g, in.indptr);
  a.rows = in.rows;
  // identity edge ids (a position view; a graph whose edges came sorted by destination):
  // the row-owned walk, which reads no edge ids (DGLMI_SOFTMAX_OWNED=0: the chunked
  // row pass + edge pass, for A/B)
  const char* owned = std::getenv("DGLMI_SOFTMAX_OWNED");
  const bool ident = (g->eid_identity & 1) != 0 && !(owned != nullptr && owned[0] == '0');
  a.eids = ident ? IdxPtr{nullptr, wide(g) ? 1 : 0} : idx(g, in.data);
  // H <= 2 there: four values per lane (DGLMI_SOFTMAX_QUAD=0: one position per lane, for A/B)
  const char* quad = std::getenv("DGLMI_SOFTMAX_QUAD");
  a.quad = !(quad != nullptr && quad[0] == '0');
  // the forward edge pass in edge-id order reads packed row statistics (DGLMI_SOFTMAX_PACK=0:
  // the two arrays, for A/B)
  const char* pack = std::getenv("DGLMI_SOFTMAX_PACK");
  a.pack = !(pack != nullptr && pack[0] == '0');
  a.coo_dst = (g->coo_src && g->coo_dst) ? g->coo_dst : nullptr;
  a.nnz = in.nnz;
  a.num_rows = in.num_rows;
  a.H = static_cast<int>(H);
  a.chunk = softmax_chunk_edges(in.nnz, H);
  return H;
}
}  // namespace

namespace {
int softmax_forward(const DGLMIGraph* graph, const DGLMIArray* logits, DGLMIArray* out, int act,
                    float slope, void* stream) {
  API_BEGIN();
  dglmi::SoftmaxArgs a;
  const int64_t H = softmax_setup(graph, logits, "logits", a);
  a.act = act;
  a.act_slope = slope;
  check_array(out, "out");
  DGLMI_CHECK(feat_numel(out) == H && out->shape[0] == logits->shape[0], "out shape");
  DGLMI_CHECK(aligned16(out->data), "out must be 16-byte aligned");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.nnz == 0) return 0;
  Scratch ws(graph, DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H), s);
  softmax_layout(a, ws.ptr, true);
  a.s = logits->data;
  a.out = out->data;
  launch_edge_softmax(a, false, s);
  check_hip(hipGetLastError(), "edge softmax forward launch");
  API_END();
}

int softmax_backward(const DGLMIGraph* graph, const DGLMIArray* out, const DGLMIArray* grad_out,
                     const DGLMIArray* logits, float slope, DGLMIArray* grad_logits, void* stream) {
  API_BEGIN();
  dglmi::SoftmaxArgs a;
  const int64_t H = softmax_setup(graph, out, "out", a);
  if (logits != nullptr) {
    check_array(logits, "logits");
    DGLMI_CHECK(feat_numel(logits) == H && logits->shape[0] == out->shape[0], "logits shape");
    DGLMI_CHECK(aligned16(logits->data), "logits must be 16-byte aligned");
    a.act = 1;
    a.act_x = logits->data;
    a.act_slope = slope;
  }
  check_array(grad_out, "grad_out");
  check_array(grad_logits, "grad_logits");
  DGLMI_CHECK(feat_numel(grad_out) == H && feat_numel(grad_logits) == H &&
                  grad_out->shape[0] == out->shape[0] && grad_logits->shape[0] == out->shape[0],
              "grad shapes");
  DGLMI_CHECK(aligned16(grad_out->data) && aligned16(grad_logits->data),
              "grads must be 16-byte aligned");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.nnz == 0) return 0;
  Scratch ws(graph, DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H), s);
  softmax_layout(a, ws.ptr, true);
  a.s = out->data;
  a.ga = grad_out->data;
  a.out = grad_logits->data;
  launch_edge_softmax(a, true, s);
  check_hip(hipGetLastError(), "edge softmax backward launch");
  API_END();
}
}  // namespace

int DGLMIEdgeSoftmaxForward(const DGLMIGraph* graph, const DGLMIArray* logits, DGLMIArray* out,
                            void* stream) {
  return softmax_forward(graph, logits, out, 0, 0.0f, stream);
}

int DGLMIEdgeSoftmaxBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                             const DGLMIArray* grad_out, DGLMIArray* grad_logits, void* stream) {
  return softmax_backward(graph, out, grad_out, nullptr, 0.0f, grad_logits, stream);
}

int DGLMIEdgeSoftmaxLeakyForward(const DGLMIGraph* graph, const DGLMIArray* logits,
                                 float negative_slope, DGLMIArray* out, void* stream) {
  return softmax_forward(graph, logits, out, 1, negative_slope, stream);
}

namespace {
// el / er of the node-logit entries: H values per row, one row per source / destination
void node_logit_args(const DGLMIGraph* g, const DGLMIArray* el, const DGLMIArray* er, int64_t H,
                     float slope, dglmi::SoftmaxArgs& a) {
  check_array(el, "el");
  check_array(er, "er");
  DGLMI_CHECK(feat_numel(el) == H && feat_numel(er) == H, "el / er must have H values per node");
  DGLMI_CHECK(el->shape[0] >= g->in_csr.num_cols && er->shape[0] >= g->in_csr.num_rows,
              "el has a row per source node, er a row per destination node");
  DGLMI_CHECK(aligned16(el->data) && aligned16(er->data), "el / er must be 16-byte aligned");
  DGLMI_CHECK(g->in_csr.nnz == 0 || g->in_csr.indices != nullptr, "in_csr.indices is required");
  a.node_l = el->data;
  a.node_r = er->data;
  a.cols = g->in_csr.indices;
  a.coo_src = a.coo_dst ? g->coo_src : nullptr;
  a.act = 1;
  a.act_slope = slope;
}
}  // namespace

int DGLMIEdgeSoftmaxNodeLogitsForward(const DGLMIGraph* graph, const DGLMIArray* el,
                                      const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                                      void* stream) {
  API_BEGIN();
  dglmi::SoftmaxArgs a;
  const int64_t H = softmax_setup(graph, out, "out", a);
  node_logit_args(graph, el, er, H, negative_slope, a);
  DGLMI_CHECK(aligned16(out->data), "out must be 16-byte aligned");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.nnz == 0) return 0;
  Scratch ws(graph, DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H), s);
  softmax_layout(a, ws.ptr, true);
  a.s = nullptr;
  a.out = out->data;
  launch_edge_softmax(a, false, s);
  check_hip(hipGetLastError(), "edge softmax (node logits) forward launch");
  API_END();
}

int DGLMIEdgeSoftmaxNodeLogitsForwardEx(const DGLMIGraph* graph, const DGLMIArray* el,
                                        const DGLMIArray* er, float negative_slope, DGLMIArray* out,
                                        DGLMIArray* row_max, DGLMIArray* row_sum, void* stream) {
  API_BEGIN();
  dglmi::SoftmaxArgs a;
  const int64_t H = softmax_setup(graph, out, "out", a);
  node_logit_args(graph, el, er, H, negative_slope, a);
  DGLMI_CHECK(aligned16(out->data), "out must be 16-byte aligned");
  check_array(row_max, "row_max");
  check_array(row_sum, "row_sum");
  DGLMI_CHECK(row_max->shape[0] == a.num_rows && feat_numel(row_max) == H && row_sum->shape[0] == a.num_rows &&
                  feat_numel(row_sum) == H,
              "row_max / row_sum must be (N_dst, H)");
  DGLMI_CHECK(aligned16(row_max->data) && aligned16(row_sum->data), "row_max / row_sum must be 16-byte aligned");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.nnz == 0) return 0;
  Scratch ws(graph, DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H), s);
  // the row statistics straight into the caller's buffers
  a.stat0 = row_max->data;
  a.stat1 = row_sum->data;
  softmax_layout(a, ws.ptr, false);
  a.s = nullptr;
  a.out = out->data;
  launch_edge_softmax(a, false, s);
  launch_sm_row_sums(a, s);
  check_hip(hipGetLastError(), "edge softmax (node logits, row statistics) forward launch");
  API_END();
}

int DGLMIEdgeSoftmaxNodeLogitsBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                                       const DGLMIArray* grad_out, const DGLMIArray* el,
                                       const DGLMIArray* er, float negative_slope,
                                       DGLMIArray* grad_logits, void* stream) {
  API_BEGIN();
  dglmi::SoftmaxArgs a;
  const int64_t H = softmax_setup(graph, out, "out", a);
  node_logit_args(graph, el, er, H, negative_slope, a);
  check_array(grad_out, "grad_out");
  check_array(grad_logits, "grad_logits");
  DGLMI_CHECK(feat_numel(grad_out) == H && feat_numel(grad_logits) == H &&
                  grad_out->shape[0] == out->shape[0] && grad_logits->shape[0] == out->shape[0],
              "grad shapes");
  DGLMI_CHECK(aligned16(grad_out->data) && aligned16(grad_logits->data),
              "grads must be 16-byte aligned");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.nnz == 0) return 0;
  Scratch ws(graph, DGLMIEdgeSoftmaxWorkspaceBytes(&graph->in_csr, H), s);
  softmax_layout(a, ws.ptr, true);
  a.s = out->data;
  a.ga = grad_out->data;
  a.out = grad_logits->data;
  launch_edge_softmax(a, true, s);
  check_hip(hipGetLastError(), "edge softmax (node logits) backward launch");
  API_END();
}

int DGLMIProjectSupported(int64_t k, int64_t n) { return dglmi::project_supported(k, n) ? 1 : 0; }

int DGLMIProject(const float* x, int64_t m, int64_t k, const float* w, int64_t w_rows,
                 int64_t w_stride_k, int64_t w_stride_n, int64_t n, const float* bias, float* y, int device,
                 void* stream) {
  API_BEGIN();
  DGLMI_CHECK(w_rows == k, "DGLMIProject: x has " + std::to_string(k) + " columns but w has " +
                               std::to_string(w_rows) + " rows");
  DGLMI_CHECK(dglmi::project_supported(k, n), "DGLMIProject: unsupported (k, n) = (" +
                                                  std::to_string(k) + ", " + std::to_string(n) + ")");
  DGLMI_CHECK(m >= 0 && x != nullptr && w != nullptr && y != nullptr, "DGLMIProject: null operand");
  DGLMI_CHECK(m == 0 || m >= 16, "DGLMIProject: tall-skinny shapes only (m >= 16 rows)");
  DGLMI_CHECK(aligned16(x) && aligned16(y) && (bias == nullptr || aligned16(bias)),
              "DGLMIProject: x, y and bias must be 16-byte aligned");
  DGLMI_CHECK(w_stride_k >= 1 && w_stride_n >= 1, "DGLMIProject: bad weight strides");
  DeviceGuard guard(device);
  dglmi::launch_project(x, m, k, w, w_stride_k, w_stride_n, n, bias, y, static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "projection launch");
  API_END();
}

int DGLMIGatAttnLogitsSupported(int64_t num_heads, int64_t head_dim) {
  return dglmi::gat_logits_supported(num_heads, head_dim) ? 1 : 0;
}

int64_t DGLMIGatAttnLogitsPartials(int64_t n_src, int64_t n_dst, int64_t num_heads, int64_t head_dim) {
  return dglmi::gat_logits_threads(n_src, n_dst, num_heads, head_dim);
}

namespace {
int check_logits_args(const float* xs, const float* xd, int64_t ns, int64_t nd, int64_t H, int64_t D,
                      const float* al, const float* ar) {
  DGLMI_CHECK(dglmi::gat_logits_supported(H, D), "DGLMIGatAttnLogits: unsupported (heads, head_dim) = (" +
                                                     std::to_string(H) + ", " + std::to_string(D) + ")");
  DGLMI_CHECK(ns >= 0 && nd >= 0 && xs != nullptr && al != nullptr && ar != nullptr,
              "DGLMIGatAttnLogits: null operand");
  DGLMI_CHECK(xd != xs || ns == nd, "DGLMIGatAttnLogits: one feature table needs n_src == n_dst");
  DGLMI_CHECK(aligned16(xs) && aligned16(xd == nullptr ? xs : xd) && aligned16(al) && aligned16(ar),
              "DGLMIGatAttnLogits: features and attention vectors must be 16-byte aligned");
  return 0;
}
}  // namespace

int DGLMIGatAttnLogits(const float* feat_src, const float* feat_dst, int64_t n_src, int64_t n_dst,
                       int64_t num_heads, int64_t head_dim, const float* attn_l, const float* attn_r,
                       float* el, float* er, int device, void* stream) {
  API_BEGIN();
  const float* xd = feat_dst == nullptr ? feat_src : feat_dst;
  check_logits_args(feat_src, xd, n_src, n_dst, num_heads, head_dim, attn_l, attn_r);
  DGLMI_CHECK(el != nullptr && er != nullptr, "DGLMIGatAttnLogits: null output");
  DeviceGuard guard(device);
  dglmi::launch_gat_logits(feat_src, xd, n_src, n_dst, static_cast<int>(num_heads),
                           static_cast<int>(head_dim), attn_l, attn_r, el, er,
                           static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "attention logits launch");
  API_END();
}

int DGLMIGatAttnLogitsBackward(const float* feat_src, const float* feat_dst, int64_t n_src, int64_t n_dst,
                               int64_t num_heads, int64_t head_dim, const float* attn_l,
                               const float* attn_r, const float* grad_el, const float* grad_er,
                               float* grad_src, float* grad_dst, float* partials, int device,
                               void* stream) {
  API_BEGIN();
  const float* xd = feat_dst == nullptr ? feat_src : feat_dst;
  check_logits_args(feat_src, xd, n_src, n_dst, num_heads, head_dim, attn_l, attn_r);
  DGLMI_CHECK(grad_el != nullptr && grad_er != nullptr && grad_src != nullptr && partials != nullptr &&
                  (xd == feat_src || grad_dst != nullptr),
              "DGLMIGatAttnLogitsBackward: null operand");
  DGLMI_CHECK(aligned16(grad_src) && aligned16(partials) && (grad_dst == nullptr || aligned16(grad_dst)),
              "DGLMIGatAttnLogitsBackward: gradients and partials must be 16-byte aligned");
  DeviceGuard guard(device);
  dglmi::launch_gat_logits_bwd(feat_src, xd, n_src, n_dst, static_cast<int>(num_heads),
                               static_cast<int>(head_dim), attn_l, attn_r, grad_el, grad_er, grad_src,
                               xd == feat_src ? nullptr : grad_dst, partials,
                               static_cast<hipStream_t>(stream));
  check_hip(hipGetLastError(), "attention logits backward launch");
  API_END();
}

int DGLMIEdgeSoftmaxLeakyBackward(const DGLMIGraph* graph, const DGLMIArray* out,
                                  const DGLMIArray* grad_out, const DGLMIArray* logits,
                                  float negative_slope, DGLMIArray* grad_logits, void* stream) {
  if (logits == nullptr) {
    g_last_error = "logits (the pre-activation input) is required";
    return -1;
  }
  return softmax_backward(graph, out, grad_out, logits, negative_slope, grad_logits, stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// The hack's extra PackedFuncs (binary_reduce.cc:398-450): the R-GCN layer
// kernels and the neighbour-access benchmark.  Relation transforms become dense
// products over node rows and every edge only gathers (hack_kernels.hip); the
// gathers run on the load-balanced reduce over relation-expanded column ids.
// ---------------------------------------------------------------------------
namespace {

DGLMIGraph plain_graph(const DGLMIGraph* g) {
  DGLMIGraph p = *g;
  p.num_col_blocks = 0;
  p.in_col_blocks = p.out_col_blocks = nullptr;
  p.in_gather_cols = p.out_gather_cols = nullptr;
  return p;
}

DGLMIGraph no_workspace() {
  DGLMIGraph z;
  std::memset(&z, 0, sizeof(z));
  return z;
}

int64_t edge_values(const DGLMIArray* norm, int64_t E, const char* name) {
  check_array(norm, name);
  const int64_t n = norm->shape[0] * feat_numel(norm);
  DGLMI_CHECK(norm->shape[0] == E && n == E, std::string(name) + " needs one value per edge");
  return n;
}

// the out-CSR regrouped by relation-expanded source row (mode 0: t * N + u, mode
// 1: u * R + t), stable: positions of a row keep their out-CSR order
struct TypedOutCsr {
  DGLMIGraph z = no_workspace();
  Scratch keys, ptr, idx, dat, rows, ws;
  DGLMICsr csr;
  TypedOutCsr(const DGLMICsr& out, const int32_t* etypes, int64_t num_typed_rows, int64_t mul,
              int mode, hipStream_t s)
      : keys(&z, out.nnz * 4, s), ptr(&z, (num_typed_rows + 1) * 4, s), idx(&z, out.nnz * 4, s),
        dat(&z, out.nnz * 4, s), rows(&z, out.nnz * 4, s),
        ws(&z, DGLMICOOToCSRDeviceWorkspaceBytes(num_typed_rows, out.nnz), s) {
    launch_typed_ids(out.rows, out.data, etypes, out.nnz, mul, mode, static_cast<int32_t*>(keys.ptr),
                     s);
    DGLMI_CHECK(DGLMICOOToCSRDevice(num_typed_rows, out.nnz, static_cast<int32_t*>(keys.ptr),
                                    out.indices, out.data, static_cast<int32_t*>(ptr.ptr),
                                    static_cast<int32_t*>(idx.ptr), static_cast<int32_t*>(dat.ptr),
                                    ws.ptr, DGLMICOOToCSRDeviceWorkspaceBytes(num_typed_rows, out.nnz),
                                    s) == 0,
                "typed CSR build");
    DGLMI_CHECK(DGLMICSRExpandRows(static_cast<int32_t*>(ptr.ptr), num_typed_rows, out.nnz,
                                   static_cast<int32_t*>(rows.ptr), s) == 0,
                "typed CSR rows");
    csr.num_rows = num_typed_rows;
    csr.num_cols = out.num_cols;
    csr.nnz = out.nnz;
    csr.indptr = static_cast<int32_t*>(ptr.ptr);
    csr.indices = static_cast<int32_t*>(idx.ptr);
    csr.data = static_cast<int32_t*>(dat.ptr);
    csr.rows = static_cast<int32_t*>(rows.ptr);
  }
};

// the graph's relation ids (DGLMIGraph.etypes) are what the entries group edges by
void rgcn_common(const DGLMIGraph* g, int64_t rows_expanded) {
  check_graph32(g, "R-GCN");
  check_csr(g->in_csr, "in_csr", true);
  check_csr(g->out_csr, "out_csr", true);
  DGLMI_CHECK(g->in_csr.nnz == g->out_csr.nnz, "in/out CSR edge counts differ");
  DGLMI_CHECK(g->in_csr.nnz == 0 || g->etypes != nullptr,
              "the graph has no edge types (DGLMIGraph.etypes is NULL)");
  DGLMI_CHECK(rows_expanded < INT32_MAX, "relations x nodes exceeds int32 indexing");
}

void check_fast_width(int64_t F) {
  DGLMI_CHECK(fast_supported(FAST_COL_MUL_EDGE_BCAST, F, F),
              "unsupported feature width " + std::to_string(F));
}

// The prepared state an entry may use (dglmi.h DGLMIRgcnState): built from the
// graph's etypes, for this relation count and source count, with the layer's bit set.
const DGLMIRgcnState* rgcn_state(const DGLMIGraph* g, int64_t R, int64_t n_src, int layer) {
  const DGLMIRgcnState* st = g->rgcn;
  if (st == nullptr || st->etypes != g->etypes || st->num_rels != R || st->num_src != n_src ||
      st->nnz != g->in_csr.nnz || !((st->layers >> layer) & 1))
    return nullptr;
  return st;
}

// The fused layer-1 walk (relation-major CSR `c` with its cached norm when the state
// was built from this norm, else edge ids + the caller's norm).
void rgcn_fused_walk(const DGLMIRgcnState* st, const DGLMICsr& c, const float* cached,
                     const float* norm, const int32_t** eids, const float** w) {
  if (st->norm != nullptr && st->norm == norm && cached != nullptr) {
    *eids = nullptr;
    *w = cached;
  } else {
    *eids = c.data;
    *w = norm;
  }
}

// A walk of the prepared in-CSR (relation-expanded columns of `layer`), with the
// cached norm streamed in position order when it was built from this norm.
DGLMICsr rgcn_in_walk(const DGLMIGraph* g, const DGLMIRgcnState* st, int layer, int64_t num_cols,
                      const float* norm, const float** w) {
  DGLMICsr walk = g->in_csr;
  walk.indices = st->in_cols[layer];
  walk.num_cols = num_cols;
  *w = norm;
  if (st->norm != nullptr && st->norm == norm && st->in_norm != nullptr) {
    walk.data = nullptr;  // edge ids = positions (run_fast reads the norm at the position)
    *w = st->in_norm;
  }
  return walk;
}

DGLMICsr rgcn_out_walk(const DGLMIRgcnState* st, int layer, const float* norm, const float** w) {
  DGLMICsr walk = st->out_typed[layer];
  *w = norm;
  if (st->norm != nullptr && st->norm == norm && st->out_norm[layer] != nullptr) {
    walk.data = nullptr;  // edge ids = positions (run_fast reads the norm at the position)
    *w = st->out_norm[layer];
  }
  return walk;
}

}  // namespace

extern "C" {

int DGLMIRgcnLayer0(const DGLMIGraph* graph, const DGLMIArray* weight,
                    const DGLMIArray* norm, DGLMIArray* ret, void* stream) {
  API_BEGIN();
  check_array(weight, "weight");
  check_array(ret, "ret");
  DGLMI_CHECK(weight->ndim == 3, "weight must be (num_rels, num_src, F)");
  const int64_t R = weight->shape[0], N = weight->shape[1], F = weight->shape[2];
  rgcn_common(graph, R * N);
  const int32_t* etypes = graph->etypes;
  const DGLMICsr& in = graph->in_csr;
  DGLMI_CHECK(in.num_cols == N, "weight rows must equal the number of source nodes");
  DGLMI_CHECK(ret->shape[0] == in.num_rows && feat_numel(ret) == F, "ret must be (num_dst, F)");
  edge_values(norm, in.nnz, "norm");
  check_fast_width(F);
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DGLMIGraph z = no_workspace(), pg = plain_graph(graph);
  if (const DGLMIRgcnState* st = rgcn_state(graph, R, N, 0)) {
    const float* w = nullptr;
    const DGLMICsr walk = rgcn_in_walk(graph, st, 0, R * N, norm->data, &w);
    run_fast(&pg, walk, FAST_COL_MUL_EDGE_BCAST, RED_SUM, weight->data, nullptr, w, nullptr,
             ret->data, F, F, s);
    return 0;
  }
  Scratch cols(&z, in.nnz * 4, s);
  launch_typed_ids(in.indices, in.data, etypes, in.nnz, N, 0, static_cast<int32_t*>(cols.ptr), s);
  DGLMICsr walk = in;
  walk.indices = static_cast<int32_t*>(cols.ptr);
  walk.num_cols = R * N;
  run_fast(&pg, walk, FAST_COL_MUL_EDGE_BCAST, RED_SUM, weight->data, nullptr, norm->data, nullptr,
           ret->data, F, F, s);
  API_END();
}

int DGLMIRgcnLayer0Backward(const DGLMIGraph* graph,
                            const DGLMIArray* grad_out, const DGLMIArray* norm,
                            DGLMIArray* grad_weight, void* stream) {
  API_BEGIN();
  check_array(grad_out, "grad_out");
  check_array(grad_weight, "grad_weight");
  DGLMI_CHECK(grad_weight->ndim == 3, "grad_weight must be (num_rels, num_src, F)");
  const int64_t R = grad_weight->shape[0], N = grad_weight->shape[1], F = grad_weight->shape[2];
  rgcn_common(graph, R * N);
  const int32_t* etypes = graph->etypes;
  const DGLMICsr& out = graph->out_csr;
  DGLMI_CHECK(out.num_rows == N, "grad_weight rows must equal the number of source nodes");
  DGLMI_CHECK(grad_out->shape[0] == graph->in_csr.num_rows && feat_numel(grad_out) == F,
              "grad_out must be (num_dst, F)");
  edge_values(norm, out.nnz, "norm");
  check_fast_width(F);
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DGLMIGraph pg = plain_graph(graph);
  if (out.nnz == 0) {
    launch_fill(grad_weight->data, R * N * F, 0.0f, s);
    return 0;
  }
  if (const DGLMIRgcnState* st = rgcn_state(graph, R, N, 0)) {
    const float* w = nullptr;
    const DGLMICsr walk = rgcn_out_walk(st, 0, norm->data, &w);
    run_fast(&pg, walk, FAST_COL_MUL_EDGE_BCAST, RED_SUM, grad_out->data, nullptr, w, nullptr,
             grad_weight->data, F, F, s);
    return 0;
  }
  TypedOutCsr typed(out, etypes, R * N, N, 0, s);
  run_fast(&pg, typed.csr, FAST_COL_MUL_EDGE_BCAST, RED_SUM, grad_out->data, nullptr, norm->data,
           nullptr, grad_weight->data, F, F, s);
  API_END();
}

namespace {
// RelGraphConv's self-loop weight (F_in x F_out) on a square graph
void check_loop_weight(const DGLMIArray* loop, int64_t K, int64_t X, const DGLMICsr& in) {
  check_array(loop, "loop_weight");
  DGLMI_CHECK(loop->ndim == 2 && loop->shape[0] == K && loop->shape[1] == X,
              "loop_weight must be (F_in, F_out)");
  DGLMI_CHECK(in.num_rows == in.num_cols, "a self-loop weight needs num_src == num_dst");
}

int rgcn_layer1_impl(const DGLMIGraph* graph, const DGLMIArray* hidden,
                     const DGLMIArray* weight, const DGLMIArray* norm, const DGLMIArray* loop,
                     const DGLMIEpilogue* epi, DGLMIArray* ret, void* stream) {
  API_BEGIN();
  check_array(hidden, "hidden");
  check_array(weight, "weight");
  check_array(ret, "ret");
  DGLMI_CHECK(weight->ndim == 3, "weight must be (num_rels, F_in, F_out)");
  const int64_t R = weight->shape[0], K = weight->shape[1], X = weight->shape[2];
  const DGLMICsr& in = graph ? graph->in_csr : DGLMICsr{};
  rgcn_common(graph, R * in.num_cols);
  const int32_t* etypes = graph->etypes;
  DGLMI_CHECK(hidden->shape[0] == in.num_cols && feat_numel(hidden) == K,
              "hidden must be (num_src, F_in)");
  DGLMI_CHECK(ret->shape[0] == in.num_rows && feat_numel(ret) == X, "ret must be (num_dst, F_out)");
  edge_values(norm, in.nnz, "norm");
  check_fast_width(X);
  const float* bias = epi ? epi->bias : nullptr;
  const float* addend = epi ? epi->addend : nullptr;
  DGLMI_CHECK(!epi || (!epi->row_mul && !epi->row_div),
              "the R-GCN epilogue takes bias and addend only");
  DGLMI_CHECK(!addend || (addend != ret->data && aligned16(addend)),
              "addend must not alias ret and must be 16-byte aligned");
  if (loop) check_loop_weight(loop, K, X, in);
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t N = in.num_cols, M = R * X;
  DGLMIGraph z = no_workspace(), pg = plain_graph(graph);
  if (const DGLMIRgcnState* fs = rgcn_state(graph, R, N, 2)) {
    if (rgcn_fused_ok(K, X, R + (loop != nullptr)) && aligned16(hidden->data) && in.nnz > 0) {
      const int32_t* eids = nullptr;
      const float* w = nullptr;
      rgcn_fused_walk(fs, fs->in_rel, fs->in_rel_norm, norm->data, &eids, &w);
      launch_rgcn_fused(false, fs->in_rel.indptr, fs->in_rel.indices, fs->in_rel.rows, eids, w,
                        hidden->data, weight->data, K * X, X, 1, ret->data, nullptr, in.num_rows, R,
                        X, s, bias, addend, loop ? loop->data : nullptr, in.num_cols);
      check_hip(hipGetLastError(), "rgcn fused layer1 launch");
      return 0;
    }
  }
  const DGLMIRgcnState* st = rgcn_state(graph, R, N, 1);
  Scratch wcat(&z, K * M * 4, s), y(&z, N * M * 4, s), cols(&z, st ? 0 : in.nnz * 4, s);
  launch_permute_rkx(weight->data, R, K, X, true, static_cast<float*>(wcat.ptr), s);
  // y[u, r * X + x] = sum_k hidden[u, k] w[r, k, x]; row u * R + r of the (N R, X) view
  launch_gemm(hidden->data, K, 1, static_cast<float*>(wcat.ptr), M, 1, static_cast<float*>(y.ptr), N,
              M, K, 1, nullptr, s);
  const float* w = norm->data;
  DGLMICsr walk = in;
  if (st) {
    walk = rgcn_in_walk(graph, st, 1, N * R, norm->data, &w);
  } else {
    launch_typed_ids(in.indices, in.data, etypes, in.nnz, R, 1, static_cast<int32_t*>(cols.ptr), s);
    walk.indices = static_cast<int32_t*>(cols.ptr);
    walk.num_cols = N * R;
  }
  // the self-loop message hidden . loop (+ the caller's addend) enters as the addend
  Scratch lt(&z, loop ? N * X * 4 : 0, s);
  if (loop) {
    launch_gemm(hidden->data, K, 1, loop->data, X, 1, static_cast<float*>(lt.ptr), N, X, K, 1,
                nullptr, s);
    if (addend) launch_add_into(static_cast<float*>(lt.ptr), addend, N * X, s);
    addend = static_cast<const float*>(lt.ptr);
  }
  const DGLMIEpilogue e2{nullptr, nullptr, bias, addend};
  run_fast(&pg, walk, FAST_COL_MUL_EDGE_BCAST, RED_SUM, static_cast<float*>(y.ptr), nullptr, w,
           nullptr, ret->data, X, X, s, (bias || addend) ? &e2 : nullptr);
  API_END();
}
}  // namespace

int DGLMIRgcnLayer1(const DGLMIGraph* graph, const DGLMIArray* hidden,
                    const DGLMIArray* weight, const DGLMIArray* norm, DGLMIArray* ret,
                    void* stream) {
  return rgcn_layer1_impl(graph, hidden, weight, norm, nullptr, nullptr, ret, stream);
}

int DGLMIRgcnLayer1Ex(const DGLMIGraph* graph, const DGLMIArray* hidden,
                      const DGLMIArray* weight, const DGLMIArray* norm,
                      const DGLMIArray* loop_weight, const DGLMIEpilogue* epilogue,
                      DGLMIArray* ret, void* stream) {
  return rgcn_layer1_impl(graph, hidden, weight, norm, loop_weight, epilogue, ret, stream);
}

namespace {
int rgcn_layer1_backward_impl(const DGLMIGraph* graph,
                              const DGLMIArray* hidden, const DGLMIArray* weight,
                              const DGLMIArray* norm, const DGLMIArray* loop,
                              const DGLMIArray* grad_out, DGLMIArray* grad_hidden,
                              DGLMIArray* grad_weight, DGLMIArray* grad_loop, void* stream) {
  API_BEGIN();
  check_array(hidden, "hidden");
  check_array(weight, "weight");
  check_array(grad_out, "grad_out");
  if (grad_hidden) check_array(grad_hidden, "grad_hidden");  // NULL (Ex only): not wanted
  check_array(grad_weight, "grad_weight");
  DGLMI_CHECK(weight->ndim == 3 && grad_weight->ndim == 3, "weights must be (num_rels, F_in, F_out)");
  const int64_t R = weight->shape[0], K = weight->shape[1], X = weight->shape[2];
  for (int i = 0; i < 3; ++i) DGLMI_CHECK(grad_weight->shape[i] == weight->shape[i], "grad_weight shape");
  const DGLMICsr& out = graph ? graph->out_csr : DGLMICsr{};
  rgcn_common(graph, R * out.num_rows);
  const int32_t* etypes = graph->etypes;
  const int64_t N = out.num_rows, M = R * X;
  DGLMI_CHECK(hidden->shape[0] == N && feat_numel(hidden) == K, "hidden must be (num_src, F_in)");
  DGLMI_CHECK(!grad_hidden || (grad_hidden->shape[0] == N && feat_numel(grad_hidden) == K),
              "grad_hidden shape");
  DGLMI_CHECK(grad_out->shape[0] == graph->in_csr.num_rows && feat_numel(grad_out) == X,
              "grad_out must be (num_dst, F_out)");
  edge_values(norm, out.nnz, "norm");
  check_fast_width(X);
  if (loop) check_loop_weight(loop, K, X, graph->in_csr);
  if (grad_loop) {
    DGLMI_CHECK(loop != nullptr, "grad_loop_weight needs loop_weight");
    check_loop_weight(grad_loop, K, X, graph->in_csr);
  }
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DGLMIGraph z = no_workspace(), pg = plain_graph(graph);
  const DGLMIRgcnState* fs = out.nnz > 0 ? rgcn_state(graph, R, N, 2) : nullptr;
  const bool fused = fs && rgcn_fused_ok(X, K, R + (loop != nullptr)) &&
                     aligned16(grad_out->data) && fs->out_typed[0].indptr;
  // the fused walk also stores grad_out as gy's last block when there is a self-loop:
  // one GEMM hidden^T . gy gives both weight gradients
  const int64_t MG = fused && loop ? M + X : M;
  const int64_t splits = gemm_splits(K, MG, N);
  const int64_t lsplits = grad_loop && !fused ? gemm_splits(K, X, N) : 1;
  Scratch gy(&z, N * MG * 4, s), gw(&z, K * MG * 4, s),
      parts(&z, std::max(splits > 1 ? splits * K * MG * 4 : 0, lsplits > 1 ? lsplits * K * X * 4 : 0),
            s);
  // grad_loop = hidden^T (K x N) . grad_out (N x X), split over N
  auto loop_weight_grad = [&]() {
    if (grad_loop)
      launch_gemm(hidden->data, 1, K, grad_out->data, X, 1, grad_loop->data, K, X, N, lsplits,
                  static_cast<float*>(parts.ptr), s);
  };
  if (fused) {
    // fused: gy rows and grad_hidden = sum_t G_t . W_t^T in one walk of the
    // relation-major out-CSR; the weight gradient from gy below
    const int32_t* eids = nullptr;
    const float* w = nullptr;
    rgcn_fused_walk(fs, fs->out_typed[0], fs->out_norm[0], norm->data, &eids, &w);
    launch_rgcn_fused(true, fs->out_typed[0].indptr, fs->out_typed[0].indices, fs->out_typed[0].rows,
                      eids, w, grad_out->data, weight->data, K * X, 1, X,
                      grad_hidden ? grad_hidden->data : nullptr, static_cast<float*>(gy.ptr), N, R,
                      K, s, nullptr, nullptr, loop ? loop->data : nullptr, graph->in_csr.num_rows);
    launch_gemm(hidden->data, 1, K, static_cast<float*>(gy.ptr), MG, 1, static_cast<float*>(gw.ptr),
                K, MG, N, splits, static_cast<float*>(parts.ptr), s);
    if (!loop) {
      launch_permute_rkx(static_cast<float*>(gw.ptr), R, K, X, false, grad_weight->data, s);
    } else {
      // gw (K x (R + 1) X) -> [R + 1][K][X]: the relation blocks, then the self-loop one
      Scratch gp(&z, (R + 1) * K * X * 4, s);
      float* p = static_cast<float*>(gp.ptr);
      launch_permute_rkx(static_cast<float*>(gw.ptr), R + 1, K, X, false, p, s);
      check_hip(hipMemcpyAsync(grad_weight->data, p, R * K * X * 4, hipMemcpyDeviceToDevice, s),
                "copy grad_weight");
      if (grad_loop)
        check_hip(hipMemcpyAsync(grad_loop->data, p + R * K * X, K * X * 4,
                                 hipMemcpyDeviceToDevice, s), "copy grad_loop_weight");
    }
    check_hip(hipGetLastError(), "rgcn fused layer1 backward launch");
    return 0;
  }
  Scratch wcat(&z, K * M * 4, s);
  launch_permute_rkx(weight->data, R, K, X, true, static_cast<float*>(wcat.ptr), s);
  // gy[u * R + t] = sum over out-edges of u with type t of norm_e * grad_out[v]
  if (const DGLMIRgcnState* st = out.nnz > 0 ? rgcn_state(graph, R, N, 1) : nullptr) {
    const float* w = nullptr;
    const DGLMICsr walk = rgcn_out_walk(st, 1, norm->data, &w);
    run_fast(&pg, walk, FAST_COL_MUL_EDGE_BCAST, RED_SUM, grad_out->data, nullptr, w, nullptr,
             static_cast<float*>(gy.ptr), X, X, s);
  } else if (out.nnz > 0) {
    TypedOutCsr typed(out, etypes, N * R, R, 1, s);
    run_fast(&pg, typed.csr, FAST_COL_MUL_EDGE_BCAST, RED_SUM, grad_out->data, nullptr, norm->data,
             nullptr, static_cast<float*>(gy.ptr), X, X, s);
  } else {
    launch_fill(static_cast<float*>(gy.ptr), N * M, 0.0f, s);
  }
  // grad_hidden = gy (N x RX) . wcat^T ; grad_wcat = hidden^T (K x N) . gy (split over N)
  if (grad_hidden)
    launch_gemm(static_cast<float*>(gy.ptr), M, 1, static_cast<float*>(wcat.ptr), 1, M,
                grad_hidden->data, N, K, M, 1, nullptr, s);
  launch_gemm(hidden->data, 1, K, static_cast<float*>(gy.ptr), M, 1, static_cast<float*>(gw.ptr), K,
              M, N, splits, static_cast<float*>(parts.ptr), s);
  launch_permute_rkx(static_cast<float*>(gw.ptr), R, K, X, false, grad_weight->data, s);
  if (loop && grad_hidden) {  // grad_hidden += grad_out . loop^T
    Scratch lt(&z, N * K * 4, s);
    launch_gemm(grad_out->data, X, 1, loop->data, 1, X, static_cast<float*>(lt.ptr), N, K, X, 1,
                nullptr, s);
    launch_add_into(grad_hidden->data, static_cast<float*>(lt.ptr), N * K, s);
  }
  loop_weight_grad();
  check_hip(hipGetLastError(), "rgcn layer1 backward launch");
  API_END();
}
}  // namespace

int DGLMIRgcnLayer1Backward(const DGLMIGraph* graph,
                            const DGLMIArray* hidden, const DGLMIArray* weight,
                            const DGLMIArray* norm, const DGLMIArray* grad_out,
                            DGLMIArray* grad_hidden, DGLMIArray* grad_weight, void* stream) {
  if (grad_hidden == nullptr) {  // the reference entry always returns both gradients
    g_last_error = "grad_hidden is NULL";
    return -1;
  }
  return rgcn_layer1_backward_impl(graph, hidden, weight, norm, nullptr, grad_out,
                                   grad_hidden, grad_weight, nullptr, stream);
}

int DGLMIRgcnLayer1BackwardEx(const DGLMIGraph* graph,
                              const DGLMIArray* hidden, const DGLMIArray* weight,
                              const DGLMIArray* norm, const DGLMIArray* loop_weight,
                              const DGLMIArray* grad_out, DGLMIArray* grad_hidden,
                              DGLMIArray* grad_weight, DGLMIArray* grad_loop_weight,
                              void* stream) {
  return rgcn_layer1_backward_impl(graph, hidden, weight, norm, loop_weight, grad_out,
                                   grad_hidden, grad_weight, grad_loop_weight, stream);
}

int DGLMIRgcnPrepare(const DGLMIGraph* graph, const DGLMIArray* norm,
                     int32_t num_rels, int32_t layers, DGLMIRgcnState* state, void* stream) {
  API_BEGIN();
  DGLMI_CHECK(state != nullptr, "null state");
  std::memset(state, 0, sizeof(*state));
  DGLMI_CHECK(num_rels >= 1, "num_rels must be >= 1");
  DGLMI_CHECK(layers >= 1 && layers <= 7,
              "layers must be a mask of 1 (layer 0), 2 (layer 1) and 4 (fused layer 1)");
  check_graph32(graph, "R-GCN");
  const DGLMICsr& in = graph->in_csr;
  const DGLMICsr& out = graph->out_csr;
  const int64_t R = num_rels, N = in.num_cols, E = in.nnz;
  rgcn_common(graph, R * N);
  const int32_t* etypes = graph->etypes;
  DGLMI_CHECK(out.num_rows == N, "out_csr rows != in_csr columns");
  if (norm != nullptr) edge_values(norm, E, "norm");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // one allocation, carved into 256-byte aligned arrays
  auto al = [](int64_t bytes) { return (bytes + 255) & ~int64_t(255); };
  const int64_t e4 = al(E * 4), ptr4 = al((R * N + 1) * 4);
  // bit 2 (fused layer 1) needs the relation-major out-CSR of layer 0 and the
  // relation-major in-CSR
  const bool want0 = (layers & 1) || (layers & 4), want1 = (layers & 2) != 0;
  const bool want_rel = (layers & 4) != 0;
  // the relation-major in-CSR keys etypes[e] * N_dst + v in int32
  DGLMI_CHECK(!want_rel || R * in.num_rows < INT32_MAX,
              "relations x destination nodes exceeds int32 indexing");
  const int nl = (want0 ? 1 : 0) + (want1 ? 1 : 0);
  const int64_t per_layer = e4 /*in cols*/ + ptr4 + 3 * e4 /*out idx, data, rows*/ +
                            (norm ? e4 : 0) /*out norm*/;
  const int64_t ptr_rel = al((R * in.num_rows + 1) * 4);
  const int64_t rel_bytes = want_rel ? ptr_rel + 3 * e4 + (norm ? e4 : 0) : 0;
  const int64_t total = e4 /*positions*/ + (norm ? e4 : 0) /*in norm*/ + nl * per_layer + rel_bytes;
  struct Owner {
    void* p = nullptr;
    ~Owner() { if (p) (void)hipFree(p); }
  } own;
  check_hip(hipMalloc(&own.p, static_cast<size_t>(std::max<int64_t>(total, 256))), "hipMalloc");
  char* cur = static_cast<char*>(own.p);
  auto take = [&](int64_t bytes) { char* r = cur; cur += bytes; return r; };
  int32_t* positions = reinterpret_cast<int32_t*>(take(e4));
  float* in_norm = norm ? reinterpret_cast<float*>(take(e4)) : nullptr;
  launch_iota_i32(positions, E, s);
  if (norm) launch_gather_f32(norm->data, in.data, E, in_norm, s);
  DGLMIGraph z = no_workspace();
  for (int layer = 0; layer < 2; ++layer) {
    if (!(layer == 0 ? want0 : want1)) continue;
    const int64_t mul = layer == 0 ? N : R;
    int32_t* cols = reinterpret_cast<int32_t*>(take(e4));
    int32_t* ptr = reinterpret_cast<int32_t*>(take(ptr4));
    int32_t* idx = reinterpret_cast<int32_t*>(take(e4));
    int32_t* dat = reinterpret_cast<int32_t*>(take(e4));
    int32_t* rows = reinterpret_cast<int32_t*>(take(e4));
    float* onorm = norm ? reinterpret_cast<float*>(take(e4)) : nullptr;
    launch_typed_ids(in.indices, in.data, etypes, E, mul, layer, cols, s);
    // the out-CSR regrouped by the same key, stable (TypedOutCsr, kept)
    const int64_t ws_bytes = DGLMICOOToCSRDeviceWorkspaceBytes(R * N, E);
    Scratch keys(&z, E * 4, s), ws(&z, ws_bytes, s);
    launch_typed_ids(out.rows, out.data, etypes, E, mul, layer, static_cast<int32_t*>(keys.ptr), s);
    DGLMI_CHECK(DGLMICOOToCSRDevice(R * N, E, static_cast<int32_t*>(keys.ptr), out.indices, out.data,
                                    ptr, idx, dat, ws.ptr, ws_bytes, s) == 0,
                std::string("typed CSR build: ") + g_last_error);
    DGLMI_CHECK(DGLMICSRExpandRows(ptr, R * N, E, rows, s) == 0,
                std::string("typed CSR rows: ") + g_last_error);
    if (norm) launch_gather_f32(norm->data, dat, E, onorm, s);
    state->in_cols[layer] = cols;
    DGLMICsr& c = state->out_typed[layer];
    c.num_rows = R * N;
    c.num_cols = out.num_cols;
    c.nnz = E;
    c.indptr = ptr;
    c.indices = idx;
    c.data = dat;
    c.rows = rows;
    state->out_norm[layer] = onorm;
  }
  if (want_rel) {
    // the in-CSR regrouped by etypes[e] * N_dst + v: one relation's rows of a tile of
    // destinations are contiguous for the fused kernel
    const int64_t nd = in.num_rows;
    int32_t* ptr = reinterpret_cast<int32_t*>(take(ptr_rel));
    int32_t* idx = reinterpret_cast<int32_t*>(take(e4));
    int32_t* dat = reinterpret_cast<int32_t*>(take(e4));
    int32_t* rows = reinterpret_cast<int32_t*>(take(e4));
    float* rnorm = norm ? reinterpret_cast<float*>(take(e4)) : nullptr;
    const int64_t ws_bytes = DGLMICOOToCSRDeviceWorkspaceBytes(R * nd, E);
    Scratch keys(&z, E * 4, s), ws(&z, ws_bytes, s);
    launch_typed_ids(in.rows, in.data, etypes, E, nd, 0, static_cast<int32_t*>(keys.ptr), s);
    DGLMI_CHECK(DGLMICOOToCSRDevice(R * nd, E, static_cast<int32_t*>(keys.ptr), in.indices, in.data,
                                    ptr, idx, dat, ws.ptr, ws_bytes, s) == 0,
                std::string("relation-major CSR build: ") + g_last_error);
    DGLMI_CHECK(DGLMICSRExpandRows(ptr, R * nd, E, rows, s) == 0,
                std::string("relation-major CSR rows: ") + g_last_error);
    if (norm) launch_gather_f32(norm->data, dat, E, rnorm, s);
    DGLMICsr& c = state->in_rel;
    c.num_rows = R * nd;
    c.num_cols = in.num_cols;
    c.nnz = E;
    c.indptr = ptr;
    c.indices = idx;
    c.data = dat;
    c.rows = rows;
    state->in_rel_norm = rnorm;
  }
  check_hip(hipGetLastError(), "rgcn prepare launch");
  state->etypes = etypes;
  state->norm = norm ? norm->data : nullptr;
  state->num_rels = num_rels;
  state->layers = layers;
  state->num_src = N;
  state->nnz = E;
  state->positions = positions;
  state->in_norm = in_norm;
  state->owner = own.p;
  own.p = nullptr;  // the state owns it now
  API_END();
}

int DGLMIRgcnRefreshNorm(const DGLMIGraph* graph, const DGLMIArray* norm, DGLMIRgcnState* state,
                         void* stream) {
  API_BEGIN();
  DGLMI_CHECK(state != nullptr && state->owner != nullptr, "state is not prepared");
  DGLMI_CHECK(state->in_norm != nullptr, "the state was prepared without a norm");
  check_graph32(graph, "R-GCN");
  DGLMI_CHECK(graph->in_csr.nnz == state->nnz, "the graph is not the state's");
  const int64_t E = state->nnz;
  edge_values(norm, E, "norm");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // every cached copy is norm permuted into a walk's position order (edge ids = data)
  launch_gather_f32(norm->data, graph->in_csr.data, E, const_cast<float*>(state->in_norm), s);
  for (int layer = 0; layer < 2; ++layer)
    if (state->out_norm[layer] != nullptr)
      launch_gather_f32(norm->data, state->out_typed[layer].data, E,
                        const_cast<float*>(state->out_norm[layer]), s);
  if (state->in_rel_norm != nullptr)
    launch_gather_f32(norm->data, state->in_rel.data, E, const_cast<float*>(state->in_rel_norm), s);
  check_hip(hipGetLastError(), "rgcn refresh norm launch");
  state->norm = norm->data;
  API_END();
}

int DGLMIRgcnRelease(DGLMIRgcnState* state) {
  API_BEGIN();
  if (state != nullptr) {
    if (state->owner != nullptr) check_hip(hipFree(state->owner), "hipFree");
    std::memset(state, 0, sizeof(*state));
  }
  API_END();
}

int DGLMINbAccess(const DGLMIGraph* graph, const DGLMIArray* feat, const int32_t* node_map,
                  const int32_t* deg_inc_node_map, int32_t times, int32_t warm_up_times,
                  double* avg_us, void* stream) {
  API_BEGIN();
  (void)node_map;          // the reference's sharding modes that read them are disabled
  (void)deg_inc_node_map;  // (binary_reduce_impl.cu:779-900); accepted and ignored
  check_graph32(graph, "NbAccess");
  check_array(feat, "feat");
  const DGLMICsr& in = graph->in_csr;
  check_csr(in, "in_csr", true);
  DGLMI_CHECK(feat->shape[0] == in.num_cols, "feat must have one row per source node");
  DGLMI_CHECK(times > warm_up_times && warm_up_times >= 0, "need times > warm_up_times >= 0");
  const int64_t F = feat_numel(feat);
  DGLMI_CHECK(fast_supported(FAST_COPY_COL, F, 1), "unsupported feature width");
  DeviceGuard guard(graph->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DGLMIGraph z = no_workspace();
  Scratch sink(&z, in.num_rows * F * 4, s);
  // destroyed on every path, a throwing check or launch included
  struct Events {
    hipEvent_t a = nullptr, b = nullptr;
    ~Events() {
      if (a) (void)hipEventDestroy(a);
      if (b) (void)hipEventDestroy(b);
    }
  } ev;
  check_hip(hipEventCreate(&ev.a), "hipEventCreate");
  check_hip(hipEventCreate(&ev.b), "hipEventCreate");
  double total = 0.0;
  for (int i = 0; i < times; ++i) {
    check_hip(hipEventRecord(ev.a, s), "hipEventRecord");
    run_fast(graph, in, FAST_COPY_COL, RED_SUM, feat->data, nullptr, nullptr, nullptr,
             static_cast<float*>(sink.ptr), F, 1, s);
    check_hip(hipEventRecord(ev.b, s), "hipEventRecord");
    check_hip(hipEventSynchronize(ev.b), "hipEventSynchronize");
    float ms = 0.0f;
    check_hip(hipEventElapsedTime(&ms, ev.a, ev.b), "hipEventElapsedTime");
    if (i >= warm_up_times) total += ms * 1e3;
  }
  if (avg_us) *avg_us = total / (times - warm_up_times);
  API_END();
}

}  // extern "C"
