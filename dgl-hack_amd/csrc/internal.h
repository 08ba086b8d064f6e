// Internal definitions shared by the C-ABI layer and the gfx950 kernels.
//
// Roles.  The reference selects kernel operands by target (src / dst / edge,
// binary_reduce_common.h:56-105) and swaps src and dst when it walks the
// reverse CSR for gradients (SwitchSrcDst, :107-121).  Here every kernel walks
// one CSR and sees operands by ROLE relative to that CSR: the row node, the
// column node, the edge, or nothing.  The host layer maps targets to roles
// for the CSR it picks (in-CSR: row = dst, col = src; out-CSR: row = src,
// col = dst), which is the same switch made explicit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dglmi.h"

namespace dglmi {

enum Role : int { ROLE_ROW = 0, ROLE_COL = 1, ROLE_EDGE = 2, ROLE_NONE = 3 };
enum Red : int { RED_SUM = 0, RED_MAX = 1, RED_MIN = 2, RED_PROD = 3, RED_NONE = 4 };
enum Op : int { OP_ADD = 0, OP_SUB = 1, OP_MUL = 2, OP_DIV = 3, OP_DOT = 4, OP_USE_LHS = 5 };

constexpr int kMaxDim = DGLMI_MAX_NDIM;

// CSR offsets (indptr) and edge ids (csr.data) as the kernels read them: int32, or
// int64 on a graph of 2^31 or more edges (DGLMIGraph.num_bits == 64; node ids stay
// int32, so indices / rows / COO arrays keep their width).  A launch-uniform flag
// picks the width on every read -- a scalar branch -- so no kernel is instantiated
// twice per index width.
struct IdxPtr {
  const void* p;
  int wide;
  __host__ __device__ __forceinline__ int64_t operator[](int64_t i) const {
    return wide ? static_cast<const int64_t*>(p)[i]
                : static_cast<int64_t>(static_cast<const int32_t*>(p)[i]);
  }
  __host__ __device__ __forceinline__ explicit operator bool() const { return p != nullptr; }
};

// Flattened broadcast description (BcastInfo, binary_reduce.h / binary_reduce.cc:96-155).
struct Bcast {
  int ndim;
  int64_t out_shape[kMaxDim], out_stride[kMaxDim];
  int64_t lhs_shape[kMaxDim], lhs_stride[kMaxDim];
  int64_t rhs_shape[kMaxDim], rhs_stride[kMaxDim];
  int64_t lhs_len, rhs_len, out_len, data_len;
};

struct Operand {
  const float* data;
  const int32_t* map;  // node map (node id -> row) or edge map (edge id -> row)
  int role;
};

// Everything a generic kernel needs; passed by value as the kernel argument.
struct EdgeArgs {
  IdxPtr indptr;           // CSR walked (rows = owners of the reduction)
  const int32_t* indices;  // column node per position
  IdxPtr eids;             // edge id per position
  const int32_t* rows;     // row per position (edge-wise kernels)
  int64_t num_rows;
  int64_t nnz;
  Operand lhs, rhs;
  float* out;              // forward: out; backward: grad buffer
  const int32_t* out_map;  // row map of `out`
  int out_role;            // ROLE_ROW (reduce to row node) or ROLE_EDGE (per edge)
  int64_t D;               // forward out features per row (x_len or bcast out_len)
  int64_t len;             // dot length (1 otherwise)
  int64_t out_rows;        // rows of `out` (bounds for the identity fill)
  // backward only
  const float* fwd_out;    // the forward output
  const float* grad_out;   // its gradient
  const int32_t* fo_map;   // row map of fwd_out/grad_out
  int fo_role;             // ROLE_COL/ROLE_ROW (node output) or ROLE_EDGE
  int want;                // 0 = grad wrt lhs, 1 = grad wrt rhs
  Bcast bc;
  // load-balanced reduce-to-row (launch_generic_lb)
  float* carry;            // workspace: num_chunks * out-row floats
  int64_t chunk;           // CSR positions per chunk
  int32_t* seg_cnt;        // num_chunks counters after the carries (segmented fixup), or null
};

// ---- device helpers ---------------------------------------------------------
template <int RED>
__device__ __forceinline__ float red_identity() {
  if constexpr (RED == RED_MAX) return -3.402823466e+38f;  // numeric_limits<float>::lowest()
  else if constexpr (RED == RED_MIN) return 3.402823466e+38f;
  else if constexpr (RED == RED_PROD) return 1.0f;
  else return 0.0f;
}

// cpu/functor.h:19-71 -- std::max / std::min tie and NaN behaviour kept.
template <int RED>
__device__ __forceinline__ float red_apply(float acc, float v) {
  if constexpr (RED == RED_MAX) return (acc < v) ? v : acc;
  else if constexpr (RED == RED_MIN) return (v < acc) ? v : acc;
  else if constexpr (RED == RED_PROD) return acc * v;
  else if constexpr (RED == RED_NONE) return v;
  else return acc + v;
}

template <int RED>
__device__ __forceinline__ float red_backward(float val, float accum) {
  if constexpr (RED == RED_MAX || RED == RED_MIN) return static_cast<float>(val == accum);
  else if constexpr (RED == RED_PROD) return accum / val;
  else return 1.0f;
}

// Rows without positions (zero in-degree) take the reducer identity.  They are
// written by a row-parallel share, not by the chunk that sees the gap: the group
// of chunk c checks rows [c·R, (c+1)·R), R = ceil(num_rows / num_chunks), and
// calls put(r) for each empty one (group-uniform; L lanes per group, L ≤ 64).
// One group filling a whole gap serialised contiguous empty rows: the ~3 M
// trailing zero-in-degree rows of M1 renumbered by degree took one group 160 ms
// (scripts/locality_probe.py).  Cost: one coalesced read of indptr per launch.
template <typename IP, typename Put>
__device__ __forceinline__ void fill_empty_rows(IP indptr, int64_t num_rows,
                                                int64_t chunk, int64_t num_chunks, int L, int lane,
                                                Put&& put) {
  const int64_t R = (num_rows + num_chunks - 1) / num_chunks;
  const int64_t r0 = chunk * R;
  const int64_t r1 = r0 + R < num_rows ? r0 + R : num_rows;
  for (int64_t base = r0; base < r1; base += L) {
    const int64_t r = base + lane;
    const bool empty = r < r1 && indptr[r] == indptr[r + 1];
    uint64_t m;
    if (L == 1) {
      m = empty ? 1u : 0u;
    } else {
      m = __ballot(empty);  // the group's lanes are converged here
      if (L < 64) m = (m >> (((threadIdx.x & 63) / L) * L)) & ((1ull << L) - 1);
    }
    while (m) {
      const int j = __builtin_ctzll(m);
      m &= m - 1;
      put(base + j);
    }
  }
}

// Segmented fixups.  A row cut into more than kFixSeg continuation chunks (a
// hub with ~10^4+ in-edges) is not folded by one group: the group of every
// kFixSeg-th continuation chunk folds its segment's carries in chunk order,
// stores the segment's partial in its own (already consumed) carry record and
// counts itself in at a per-row counter; the group that arrives last folds the
// row head and the segment partials in segment order.  Deterministic (the same
// association on every run), and no group waits on another.  One group folding
// 39 K carries made a 20 M-edge star's copy_u sum 5.4 ms (0.8 ms spread over
// 1 M rows; scripts/hub_probe.py).  Counters live after the carries in the
// workspace, one per chunk, zeroed by the reduce kernel that precedes the fixup.
// Like fill_empty_rows, seg_arrive_last needs the L lanes of a group inside ONE
// wavefront (L <= 64: lane 0's counter value reaches the others by a shuffle);
// the templated kernels static_assert it and the generic ones cap L at 64
// (kernels_generic.hip kMaxLaneBits).
constexpr int64_t kFixSeg = 32;
__device__ __forceinline__ bool seg_arrive_last(int32_t* cnt, int64_t nseg, int L, int lane) {
  __threadfence();  // release: this group's partial, past its XCD's L2
  int old = 0;
  if (lane == 0) old = atomicAdd(cnt, 1);
  if (L > 1) old = __shfl(old, 0, L);
  const bool last = old == static_cast<int>(nseg - 1);
  if (last) __threadfence();  // acquire: the other segments' partials
  return last;
}

// binary_reduce_common.h:131-213
template <int OP>
__device__ __forceinline__ float op_apply(const float* l, const float* r, int64_t len) {
  if constexpr (OP == OP_ADD) return l[0] + r[0];
  else if constexpr (OP == OP_SUB) return l[0] - r[0];
  else if constexpr (OP == OP_MUL) return l[0] * r[0];
  else if constexpr (OP == OP_DIV) return l[0] / r[0];
  else if constexpr (OP == OP_USE_LHS) return l[0];
  else {
    float out = 0.0f;
    for (int64_t i = 0; i < len; ++i) out += l[i] * r[i];
    return out;
  }
}
template <int OP>
__device__ __forceinline__ float op_grad_lhs(float l, float r) {
  if constexpr (OP == OP_MUL || OP == OP_DOT) return r;
  else if constexpr (OP == OP_DIV) return 1.0f / r;
  else return 1.0f;
}
template <int OP>
__device__ __forceinline__ float op_grad_rhs(float l, float r) {
  if constexpr (OP == OP_ADD) return 1.0f;
  else if constexpr (OP == OP_SUB) return -1.0f;
  else if constexpr (OP == OP_MUL || OP == OP_DOT) return l;
  else if constexpr (OP == OP_DIV) return -l / (r * r);
  else return 0.0f;
}

__device__ __forceinline__ int64_t resolve(const Operand& o, int64_t row, int64_t col,
                                           int64_t eid) {
  int64_t id = o.role == ROLE_ROW ? row : (o.role == ROLE_COL ? col : (o.role == ROLE_EDGE ? eid : 0));
  if (o.map && o.role != ROLE_NONE) id = o.map[id];
  return id;
}

// Set the calling thread's DGLMIGetLastError() message (capi.cpp), for the C
// entry points defined outside capi.cpp.
void set_last_error(const char* msg);

// ---- host-side launchers (defined in the .hip files) ------------------------
void launch_fill(float* out, int64_t n, float value, hipStream_t s);
void launch_fill_i32(int32_t* out, int64_t n, int32_t value, hipStream_t s);
// out[r, :] = out[r, :] * row_mul[r] / row_div[r] + bias + addend[r, :] (each optional)
void launch_epilogue(float* out, int64_t rows, int64_t F, const float* row_mul,
                     const float* row_div, const float* bias, const float* addend,
                     hipStream_t s);

// Generic forward: reduce to row nodes (out_role == ROLE_ROW) or per edge.
void launch_generic_forward(int op, int red, bool bcast, const EdgeArgs& a, hipStream_t s);
// Generic backward for one operand (a.want), reduce to row nodes or per edge.
void launch_generic_backward(int op, int red, bool bcast, const EdgeArgs& a, hipStream_t s);

// Load-balanced reduce-to-row for every op / reducer / broadcast (fixed chunks
// of CSR positions + carry fixup).  Needs a.rows; returns false (nothing
// launched) when the output row is too wide for it.
bool generic_lb_supported(int64_t out_row_len);
void launch_generic_lb(int op, int red, bool bcast, bool bwd, const EdgeArgs& a, hipStream_t s);

// Per-edge outputs (kernels_sddmm.hip).  Roles are relative to the in-CSR:
// ROLE_ROW = destination node, ROLE_COL = source node, ROLE_EDGE = edge id.
struct SddmmArgs {
  const int32_t* rows;  // destination node per item
  const int32_t* cols;  // source node per item
  IdxPtr eids;          // edge id per item; NULL: item index == edge id (COO order)
  int64_t nnz;
  const float* lhs;
  const float* rhs;
  int lhs_role, rhs_role;
  float* out;           // forward: (E, D); backward: (E, D * len) gradient rows
  const float* go;      // backward: grad of the forward output
  int go_role;          // ROLE_EDGE (reducer none) or ROLE_ROW (reducer sum)
  int want;             // backward: 0 = lhs, 1 = rhs
  int64_t D, len;       // output features, dot length (1 otherwise)
};
bool sddmm_supported(int op, bool bwd, int64_t D, int64_t len);
void launch_sddmm(int op, bool bwd, const SddmmArgs& a, hipStream_t s);

// Fused edge softmax (kernels_softmax.hip).
struct SoftmaxArgs {
  IdxPtr indptr;           // in-CSR
  const int32_t* rows;
  IdxPtr eids;
  const int32_t* coo_dst;  // optional: edge-id order for the per-edge pass
  int64_t nnz;
  int64_t num_rows;
  int H;                   // values per edge
  const float* s;          // forward: logits; backward: the softmax output
  const float* ga;         // backward: gradient wrt the output
  float* stat0;            // forward: row max m; backward: row sum S (num_rows x H)
  float* stat1;            // forward: row sum of exp l
  float* out;              // forward: softmax; backward: gradient wrt the logits
  float* carry;            // num_chunks x 2H
  int64_t chunk;
  int32_t* seg_cnt;        // num_chunks counters after the carries (segmented fixup), or null
  // GATConv's leaky_relu -> edge_softmax pair in one pass (act != 0): the forward reads the
  // pre-activation logits x and takes the softmax of leaky(x) = x > 0 ? x : x * slope; the
  // backward multiplies its gradient by leaky'(x) = x > 0 ? 1 : slope, x read from act_x
  // (torch's leaky_relu / leaky_relu_backward, the same operations in the same order)
  const float* act_x;
  float act_slope;
  int act;
  // GATConv's u_add_v -> leaky_relu -> edge_softmax (node_l != null): the logit of the
  // edge at in-CSR position p is node_l[cols[p]] + node_r[rows[p]] (H values each; the
  // SDDMM's lhs + rhs), computed where the softmax reads it -- forward, and the backward's
  // leaky_relu mask -- so the per-edge logits are never stored
  const float* node_l;
  const float* node_r;
  const int32_t* cols;     // in-CSR indices (node_l mode)
  const int32_t* coo_src;  // with coo_dst: the edge-id-order pass's source per edge
  int quad;                // H <= 4 on the row-owned walk: four values per lane (16-B loads)
  // the forward edge pass in edge-id order: each row's (max, sum) side by side (2H floats),
  // packed after the row pass (one request per edge instead of two); null: stat0 / stat1
  int pack;
  float* stat_pk;
};
bool softmax_supported(int64_t H);

// Tall-skinny projection Y = X W (+ bias) on MFMA (kernels_project.hip): X (M, K)
// row-major, W (K, N) with strides (swk, swn), Y (M, N) row-major.
bool project_supported(int64_t K, int64_t N);
void launch_project(const float* X, int64_t M, int64_t K, const float* W, int64_t swk, int64_t swn,
                    int64_t N, const float* bias, float* Y, hipStream_t s);
int64_t softmax_chunk_edges(int64_t nnz, int64_t H);
// eids NULL (identity edge ids): the row-owned walk (one read, one write per value);
// its carries need this many bytes after the statistics
int64_t softmax_owned_carry_bytes(int64_t nnz, int64_t H);
void launch_edge_softmax(const SoftmaxArgs& a, bool backward, hipStream_t s);
// after a forward: a.stat0 = each row's max, a.stat1 = its sum of exp(s - max) (the
// row-owned walk leaves 1 / sum there: inverted in place; rows without edges: 0 and
// 1 / 0 = inf -- never read by an edge)
void launch_sm_row_sums(const SoftmaxArgs& a, hipStream_t s);

// Load-balanced reduce-to-row kernels (kernels_spmm.hip).
enum FastKind : int {
  FAST_COPY_COL = 0,    // v = X[col]
  FAST_COPY_EDGE = 1,   // v = E[eid]
  FAST_COL_MUL_EDGE = 2,        // v = X[col] * E[eid]            (same feature shape)
  FAST_COL_MUL_EDGE_BCAST = 3,  // v = X[col, h, :] * E[eid, h]   (E broadcast over the last dim)
  FAST_COL_TIE = 4,     // v = XR[row] == W[col] ? X[col] : 0  (max / min gradient, tie mask)
  FAST_COL_MUL_POS = 5, // v = X[col] * W[p], one weight per position (identity edge ids; sum)
};
struct FastArgs {
  IdxPtr indptr;
  const int32_t* rows;
  const int32_t* indices;
  IdxPtr eids;
  int64_t nnz;
  int64_t num_rows;     // rows owned (out rows 0..num_rows-1 written)
  const float* x;       // column-node or edge features
  const float* w;       // edge features (mul kinds)
  const int32_t* x_map; // optional row maps
  const int32_t* w_map;
  float* out;
  int64_t F;            // features per output row
  int64_t head_dim;     // bcast: features per head (E has F / head_dim values per edge)
  float* carry;         // workspace: num_chunks * F floats
  int32_t* seg_cnt;     // num_chunks counters after the carries (segmented fixup), or null
  int64_t chunk;        // edges per chunk
  // optional fused epilogue (sum only): out = acc * row_mul[r] / row_div[r] + bias + addend[r]
  const float* row_mul;
  const float* row_div;
  const float* bias;
  const float* addend;
  // copy_u sum: `indices` carries cold-row marks in bit 31 (DGLMIKernelMarkColdColumns);
  // marked rows are gathered non-temporally
  int marked;
  const float* xr;      // FAST_COL_TIE: the reduce's input, one row per walk row
  int64_t num_cols;     // rows of the gathered table (policy-probe bound check)
};
int64_t fast_chunk_edges(int64_t nnz, int64_t F);
int64_t fast_workspace_bytes(int64_t nnz, int64_t F);  // carries + counters
int64_t fast_carry_bytes(int64_t nnz, int64_t F);      // offset of the counters
// Returns false if the shape is not supported by the fast path.
bool fast_supported(int kind, int64_t F, int64_t head_dim);
void launch_fast_reduce(int kind, int red, const FastArgs& a, hipStream_t s);  // needs a.indptr
// out_cols[p] = cols[p] | (col_deg(cols[p]) < thresh ? 1 << 31 : 0), col_deg from deg_indptr
void launch_mark_cold(const int32_t* cols, int64_t nnz, IdxPtr deg_indptr, int32_t thresh,
                      int32_t* out_cols, hipStream_t s);
// row widths whose launch config has a marked variant (L >= 16 lanes, one float4 each)
inline bool fast_marked_supported(int64_t F) { return F > 32 && F <= 256 && F % 4 == 0; }
// tables smaller than this stay on the plain path (they fit the Infinity Cache)
constexpr int64_t kMarkedMinTableBytes = int64_t(256) << 20;

// Fused GAT (kernels_gat.hip).
struct GatArgs {
  const int32_t* indptr;
  const int32_t* rows;
  const int32_t* indices;
  int64_t nnz;
  int64_t num_rows;
  int H, D;
  int64_t F;  // H * D
  float slope;
  const float* ft;  // (N_src, H, D)
  const float* el;  // (N_src, H)
  const float* er;  // (N_dst, H)
  float* out;       // (N_dst, H, D)
  float* m;         // (N_dst, H)
  float* l;         // (N_dst, H)
  const float* go;  // grad_out (N_dst, H, D)
  const float* fo;  // forward out (N_dst, H, D)
  const float* m_in;
  const float* l_in;
  float4* stats;    // (N_dst, H): {er, m, 1/l, delta}
  float* g_er;
  float* g_el;
  float* g_ft;
  float* carry;
  int32_t* seg_cnt;  // num_chunks counters after the carries (segmented fixup), or null
  int64_t chunk;
  // column-blocked launches (one launch per block of gathered rows):
  int raw;          // forward: leave (m, l, acc) unnormalised (merged afterwards)
  int accumulate;   // backward: add into g_er / g_ft / g_el instead of overwriting
  int skip_stats;   // backward (dst side): stats already written by an earlier block
  int o32;          // every gathered row offset (ft, el, grad_out, stats) < 2^31 elements
  // edge-position backward (DGLMIGraph.gat_edge_pos): the source-side walk stores every
  // edge's grad_er term at t[(t_off + position) * H + h]; NULL = not stored
  float* t;
  int64_t t_off;
  // slope aggregates (DGLMIFusedGatForwardEx): the forward writes, per destination row
  // and head, lf = sum_in a_e lrelu'(pre_e) ft[u] (N_dst, H, D) and ls = sum_in a_e
  // lrelu'(pre_e) (N_dst, H); with them the backward's k_gat_stats also writes grad_er
  // and no destination-side walk runs.  NULL = not kept.
  float* lf;
  float* ls;
  // attention dropout.  drop = 0: off.  drop = 1 (DGLMIFusedGatDropout*, hashed): edge e,
  // head h keeps its weight, scaled by drop_scale, when gat_head_keep(gat_edge_key(seed,
  // eid), h, drop_thresh) (16-bit threshold, round(p 2^16)).  drop = 2 (DGLMIFusedGatKeep*,
  // the caller's mask): bit h of drop_bits[eid] -- one word per edge id of drop_width bits
  // (8, 16 or 32: the narrowest that holds H, so C3's 114.6 M edges at H = 8 take 115 MB,
  // Infinity-Cache resident, for the walks' random reads), drawn by the caller (GATConv:
  // its nn.Dropout) -- scaled by drop_scale.  The walk's edge ids in `eids` (its CSR's data).
  int drop;
  uint32_t drop_thresh;
  float drop_scale;
  uint64_t drop_seed;
  const void* drop_bits;
  int drop_width;
  // drop_pos: the keep words are in this walk's position order, at drop_bits[drop_off +
  // position] (coalesced; the caller gathers them once per direction, column blocks
  // concatenated in block order) instead of at drop_bits[edge id] (a random read per edge)
  int drop_pos;
  int64_t drop_off;
  // drop_rng = 1 (DGLMIFusedGatDraw*; drop = 1's instances): edge e, head h is kept when
  // torch's fused dropout over the (E, H) attention tensor keeps element e * H + h --
  // its Philox draw recomputed from (rng_seed, rng_ctr = offset / 4, rng_threads = the
  // draw's grid x 256, rng_vec) by gat_draw_keep, kept below rng_keep = float(1 - p);
  // rng_shift = log2(rng_threads) when that is a power of two (the capped grid), else -1
  int drop_rng;
  int rng_vec;
  int rng_shift;
  float rng_keep;
  uint64_t rng_seed;
  uint64_t rng_ctr;
  int64_t rng_threads;
  const int32_t* eids;
};
// Philox4x32-10 (Salmon et al., SC'11 "Random123"): the generator torch draws its fused
// dropout from on this build (hiprand / rocrand's philox4x32_10).  Counter (x, y) = the
// draw index on top of offset / 4, (z, w) = the drawing thread's subsequence; the key is
// the 64-bit seed, bumped by the Weyl constants between the ten rounds.
__host__ __device__ __forceinline__ uint32_t philox_mulhi(uint32_t a, uint32_t b) {
  return static_cast<uint32_t>((static_cast<uint64_t>(a) * b) >> 32);
}
struct Philox4 {
  uint32_t x, y, z, w;
};
__host__ __device__ __forceinline__ Philox4 philox4x32_10(Philox4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = philox_mulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = philox_mulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = Philox4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// torch's fused dropout kernel (256-thread blocks, grid capped at CUs x 8, one uniform4
// draw per thread per pass; scripts/philox_probe.py pins the mapping on this build) as a
// function of the element index i: which thread t drew it, in which of that thread's
// draws j, which component.  vec 4 (numel % 4 == 0): four consecutive elements per thread
// and pass; vec 2: two, a fresh draw every pass (components x, y); vec 1 (the unrolled
// scalar kernel): element i is thread i % T's, pass q = i / T, draw q / 4, component q % 4.
struct DrawSlot {
  int64_t t, j;
  int comp;
};
__host__ __device__ __forceinline__ DrawSlot dropout_draw_slot(int64_t i, int vec, int64_t T, int shift) {
  DrawSlot s;
  const int64_t c = vec == 4 ? i >> 2 : vec == 2 ? i >> 1 : i;
  int64_t q, t;
  if (shift >= 0) {
    q = c >> shift;
    t = c & (T - 1);
  } else {
    q = c / T;
    t = c - q * T;
  }
  s.t = t;
  if (vec == 4) {
    s.j = q;
    s.comp = static_cast<int>(i & 3);
  } else if (vec == 2) {
    s.j = q;
    s.comp = static_cast<int>(i & 1);
  } else {
    s.j = q >> 2;
    s.comp = static_cast<int>(q & 3);
  }
  return s;
}
__host__ __device__ __forceinline__ Philox4 dropout_draw(uint64_t seed, uint64_t ctr, const DrawSlot& s) {
  const uint64_t c = ctr + static_cast<uint64_t>(s.j);
  const uint64_t t = static_cast<uint64_t>(s.t);
  return philox4x32_10(Philox4{static_cast<uint32_t>(c), static_cast<uint32_t>(c >> 32),
                               static_cast<uint32_t>(t), static_cast<uint32_t>(t >> 32)},
                       static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
}
// rocrand's uniform: 2^-32 + v 2^-32 (exact with or without contraction: the product is a
// power-of-two scaling), kept when below the keep probability
__host__ __device__ __forceinline__ bool dropout_draw_kept(const Philox4& r, int comp, float keep) {
  const uint32_t v = comp == 0 ? r.x : comp == 1 ? r.y : comp == 2 ? r.z : r.w;
  return 2.3283064365386963e-10f + static_cast<float>(v) * 2.3283064365386963e-10f < keep;
}
// mask[i] = kept(i) for i < n: the draw's whole mask (DGLMIDropoutDrawMask: tests, and the
// self-check against torch.native_dropout before the fused route trusts the mapping)
void launch_dropout_draw_mask(uint64_t seed, uint64_t ctr, int64_t threads, int vec, int shift, float keep,
                              int64_t n, uint8_t* mask, hipStream_t s);
// out[p H + h] = drop_scale if the draw keeps element eids[p] H + h, else 0, p < n (a.H
// heads <= 32, a.rng_* set; eids NULL = identity): the draw's output on a tensor of ones
// in a walk's position order (GATConv's composition: dropout(a) on the position view)
// apply = true: out[p H + h] *= that factor instead (dropout applied in place)
void launch_dropout_draw_scale(const GatArgs& a, const int32_t* eids, int64_t n, float* out, bool apply,
                               hipStream_t s);
// The dropout mask's hash (mirrored in numpy by dgl.kernel.gat_dropout_keep for the
// tests): one key per edge -- a 32-bit avalanche mix of the edge id keyed by the seed's
// low half, xor the high half -- then, per PAIR of heads, a one-multiply finish of
// key + (pair + 1) * golden ratio whose low / high 16 bits decide heads 2j / 2j + 1
// (kept when >= the 16-bit threshold).  Two multiplies per edge plus one per pair of
// heads (the staging lane's VALU is what the dropout walks pay for), and no eid * H
// product (it wrapped at 2^32 edge-heads).
__host__ __device__ __forceinline__ uint32_t gat_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ uint32_t gat_edge_key(uint64_t seed, uint32_t eid) {
  return gat_mix32(eid ^ static_cast<uint32_t>(seed)) ^ static_cast<uint32_t>(seed >> 32);
}
__host__ __device__ __forceinline__ uint32_t gat_pair_bits(uint32_t key, int pair) {
  uint32_t x = key + static_cast<uint32_t>(pair + 1) * 0x9e3779b9u;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}
__host__ __device__ __forceinline__ bool gat_head_keep(uint32_t key, int h, uint32_t thresh16) {
  return ((gat_pair_bits(key, h >> 1) >> (16 * (h & 1))) & 0xffffu) >= thresh16;
}
bool gat_supported(int64_t H, int64_t D);
// bits[e] = OR over h < H of (table[e * H + h] != 0) << h, e < n (H <= width <= 32): a
// dropout output table (E, H) in edge-id order packed to one keep word of `width` bits
// (8, 16 or 32) per edge (drop = 2)
void launch_gat_keep_bits(const float* table, int64_t n, int H, void* bits, int width, hipStream_t s);
void launch_gat_keep_bits_mask(const uint8_t* mask, int64_t n, int H, void* bits, int width, hipStream_t s);
// out[i] = keep[index[i]], i < n, words of `width` bits: edge-id keep words into a walk's
// position order (index = the walk CSR's edge ids)
void launch_gat_keep_gather(const void* keep, int width, const int32_t* index, int64_t n, void* out,
                            hipStream_t s);
int64_t gat_chunk_edges(int64_t nnz);
void launch_gat_forward(const GatArgs& a, hipStream_t s);
void launch_gat_backward_dst(const GatArgs& a, hipStream_t s);
void launch_gat_backward_src(const GatArgs& a, hipStream_t s);
// stats[v, h] = {er, m, 1/l, <grad_out[v,h,:], out[v,h,:]>} for every destination row
// (dense; replaces the destination-side walk's stats when gat_edge_pos is given); with
// a.lf / a.ls (the forward's slope aggregates) also grad_er = <grad_out, lf> - delta ls
void launch_gat_stats(const GatArgs& a, hipStream_t s);
// out[r] = merge over blocks b of the unnormalised partials (out_part[b], m_part[b],
// l_part[b]), normalised; m / l of the merged softmax (blocks in order); lf / ls from
// lf_part / ls_part the same way (all four NULL: none)
void launch_gat_merge(const float* out_part, const float* m_part, const float* l_part, int nb,
                      int64_t num_rows, int H, int D, float* out, float* m, float* l, hipStream_t s,
                      const float* lf_part = nullptr, const float* ls_part = nullptr,
                      float* lf = nullptr, float* ls = nullptr);
// l[i] = m[i] + log(l[i]) for i < n (one log-sum-exp per row and head)
void launch_gat_fold_lse(const float* m, float* l, int64_t n, hipStream_t s);
// GATConv's attention logits el = (xs * al).sum(-1), er = (xd * ar).sum(-1) (xs, xd (n, H,
// D) row-major, al / ar (H, D); xd == xs: one table) and their backward (gs = gel al, gd =
// ger ar -- one table: gs = gel al + ger ar, gd unused; part: gat_logits_threads x 8
// floats of parameter-gradient partials).  Supported: D % 4 == 0, D / 4 a power of two
// <= 16, H D / 4 dividing 256.
bool gat_logits_supported(int64_t H, int64_t D);
int64_t gat_logits_threads(int64_t ns, int64_t nd, int64_t H, int64_t D);
void launch_gat_logits(const float* xs, const float* xd, int64_t ns, int64_t nd, int H, int D,
                       const float* al, const float* ar, float* el, float* er, hipStream_t s);
void launch_gat_logits_bwd(const float* xs, const float* xd, int64_t ns, int64_t nd, int H, int D,
                           const float* al, const float* ar, const float* gel, const float* ger,
                           float* gs, float* gd, float* part, hipStream_t s);

// R-GCN C entries (hack_kernels.hip): relation-expanded ids (mode 0: etypes[eid] *
// mul + id, mode 1: id * mul + etypes[eid]; eids NULL = position), the relation
// weight layout (R, K, X) <-> (K, R * X), and C (M x N, row-major) = A . B with A,
// B by (row, col) strides, the reduction split `splits` ways through `partials`
// (splits * M * N floats) when splits > 1 (gemm_splits picks it).
void launch_typed_ids(const int32_t* ids, const int32_t* eids, const int32_t* etypes, int64_t nnz,
                      int64_t mul, int mode, int32_t* out, hipStream_t s);
void launch_permute_rkx(const float* w, int64_t R, int64_t K, int64_t X, bool to_cat, float* out,
                        hipStream_t s);
// Fused R-GCN layer 1 (hack_kernels.hip k_rgcn_fused): the relation-major CSR (rows
// t * num_rows + v, `rows` = its COO rows, eids NULL = w by position), gathered table T
// of 64-float rows, weights W[t][k][n] by strides; out (num_rows x out_w); bwd also
// writes gy (num_rows x R * 64).  loop_w (same k / n strides): one more matrix applied
// to the tile's own rows of T (RelGraphConv's self-loop; square graphs).
// rgcn_fused_ok: the shapes it takes (R counts the self-loop matrix too).
bool rgcn_fused_ok(int64_t gathered_w, int64_t out_w, int64_t R);
void launch_rgcn_fused(bool bwd, const int32_t* ptr, const int32_t* cols, const int32_t* rows,
                       const int32_t* eids, const float* w, const float* T, const float* W,
                       int64_t ws_t, int64_t ws_k, int64_t ws_n, float* out, float* gy,
                       int64_t num_rows, int64_t R, int64_t out_w, hipStream_t s,
                       const float* bias = nullptr, const float* addend = nullptr,
                       const float* loop_w = nullptr, int64_t t_rows = -1);
// out[i] += a[i], i < n
void launch_add_into(float* out, const float* a, int64_t n, hipStream_t s);
// out[p] = v[idx[p]]; out[p] = p
void launch_gather_f32(const float* v, const int32_t* idx, int64_t n, float* out, hipStream_t s);
void launch_iota_i32(int32_t* out, int64_t n, hipStream_t s);
int64_t gemm_splits(int64_t M, int64_t N, int64_t K);
void launch_gemm(const float* A, int64_t a_rs, int64_t a_cs, const float* B, int64_t b_rs,
                 int64_t b_cs, float* C, int64_t M, int64_t N, int64_t K, int64_t splits,
                 float* partials, hipStream_t s);

}  // namespace dglmi
