/*
 * oracle/dgl_ref.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the reference's CPU kernel semantics for the
 * g-SpMM / g-SDDMM ("binary reduce" / "copy reduce") path of ydwu4/dgl-hack
 * (a DGL 0.4 fork).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.
 *
 * The reference library itself cannot be built here: every submodule
 * (minigun, dmlc-core, dlpack) is empty, so this file restates
 * the algorithm from the reference sources, function by function:
 *
 *   ref_binary_reduce      src/kernel/cpu/binary_reduce_impl.h:24-52 (UDF),
 *                          :56-109 (broadcast UDF, Unravel/Ravel),
 *                          :147-173 (out-CSR traversal, edge mapping := csr.data),
 *                          src/kernel/binary_reduce_impl.h:31-64 (identity fill),
 *                          src/kernel/binary_reduce.cc:96-155 (CalcBcastInfo),
 *                          :214-219 (NeedSwitchOrder), :295-336 (dispatch)
 *   reducers               src/kernel/cpu/functor.h:19-71, identities
 *                          src/kernel/binary_reduce_common.h:444-485
 *   binary ops             src/kernel/binary_reduce_common.h:131-213
 *   ref_backward           src/kernel/cpu/backward_binary_reduce_impl.h:22-161
 *                          (UDF), :212-245 (in-CSR traversal with src/dst
 *                          switched), src/kernel/binary_reduce_impl.h:119-222
 *   ref_coo_to_csr         src/array/cpu/spmat_op_impl_coo.cc:230-283
 *   ref_csr_transpose      src/array/cpu/spmat_op_impl.cc:323-369
 *
 * The minigun traversal (external, un-vendored, commit unknown) is restated
 * from its call sites: for every CSR row r (OpenMP-parallel) and every
 * position j in [indptr[r], indptr[r+1]) it calls ApplyEdge(r, indices[j], j).
 * With nthreads == 1 the summation order is deterministic (row asc, then CSR
 * position asc); with more threads it reproduces the reference's `omp atomic`
 * scatter (`omp critical` for max/min) and is used as the CPU baseline.
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

enum { T_SRC = 0, T_DST = 1, T_EDGE = 2, T_NONE = 3 };
enum { R_SUM = 0, R_MAX, R_MIN, R_PROD, R_NONE };
enum { O_ADD = 0, O_SUB, O_MUL, O_DIV, O_DOT, O_USE_LHS };
#define MAXDIM 8

static int parse_reducer(const char* s) {
  if (!strcmp(s, "sum") || !strcmp(s, "mean")) return R_SUM; /* mean -> sum, REDUCER_SWITCH */
  if (!strcmp(s, "max")) return R_MAX;
  if (!strcmp(s, "min")) return R_MIN;
  if (!strcmp(s, "prod")) return R_PROD;
  if (!strcmp(s, "none")) return R_NONE;
  return -1;
}
static int parse_op(const char* s) {
  if (!strcmp(s, "add")) return O_ADD;
  if (!strcmp(s, "sub")) return O_SUB;
  if (!strcmp(s, "mul")) return O_MUL;
  if (!strcmp(s, "div")) return O_DIV;
  if (!strcmp(s, "dot")) return O_DOT;
  if (!strcmp(s, "use_lhs")) return O_USE_LHS;
  return -1;
}

/* binary_reduce_common.h:131-213 */
static inline float op_call(int op, const float* l, const float* r, int64_t len) {
  switch (op) {
    case O_ADD: return l[0] + r[0];
    case O_SUB: return l[0] - r[0];
    case O_MUL: return l[0] * r[0];
    case O_DIV: return l[0] / r[0];
    case O_USE_LHS: return l[0];
    default: {
      float out = 0;
      for (int64_t i = 0; i < len; ++i) out += l[i] * r[i];
      return out;
    }
  }
}
static inline float op_bwd_lhs(int op, float l, float r) {
  switch (op) {
    case O_MUL: case O_DOT: return r;
    case O_DIV: return 1.0f / r;
    default: return 1.0f; /* add, sub, use_lhs */
  }
}
static inline float op_bwd_rhs(int op, float l, float r) {
  switch (op) {
    case O_ADD: return 1.0f;
    case O_SUB: return -1.0f;
    case O_MUL: case O_DOT: return l;
    case O_DIV: return -l / (r * r);
    default: return 0.0f; /* use_lhs */
  }
}
/* identity values: binary_reduce_common.h:444-485 */
static float red_zero(int red) {
  switch (red) {
    case R_MAX: return -FLT_MAX;  /* numeric_limits<float>::lowest() */
    case R_MIN: return FLT_MAX;
    case R_PROD: return 1.0f;
    default: return 0.0f;
  }
}
/* std::max(a, b) = (a < b) ? b : a and std::min(a, b) = (b < a) ? b : a, exactly
 * as <algorithm> defines them (cpu/functor.h:33,44 call them as
 * std::max(*addr, val)): a NaN `val` never replaces the accumulator, a NaN
 * accumulator is kept. */
static inline float std_max(float a, float b) { return (a < b) ? b : a; }
static inline float std_min(float a, float b) { return (b < a) ? b : a; }

/* cpu/functor.h:19-71 */
static inline void red_call(int red, float* addr, float val, int par) {
  switch (red) {
    case R_SUM:
      if (par) {
#pragma omp atomic
        *addr += val;
      } else {
        *addr += val;
      }
      break;
    case R_MAX:
      if (par) {
#pragma omp critical
        *addr = std_max(*addr, val);
      } else {
        *addr = std_max(*addr, val);
      }
      break;
    case R_MIN:
      if (par) {
#pragma omp critical
        *addr = std_min(*addr, val);
      } else {
        *addr = std_min(*addr, val);
      }
      break;
    case R_PROD:
      if (par) {
#pragma omp atomic
        *addr *= val;
      } else {
        *addr *= val;
      }
      break;
    default: *addr = val;
  }
}
static inline float red_bwd(int red, float val, float accum) {
  switch (red) {
    case R_MAX: case R_MIN: return (float)(val == accum);
    case R_PROD: return accum / val;
    default: return 1.0f;
  }
}
static inline int64_t sel(int tgt, int64_t src, int64_t eid, int64_t dst) {
  switch (tgt) {
    case T_SRC: return src;
    case T_DST: return dst;
    case T_EDGE: return eid;
    default: return 0;
  }
}

/* ---- broadcast info: binary_reduce.cc:96-155 ------------------------------ */
typedef struct {
  int ndim;
  int64_t lhs_shape[MAXDIM], rhs_shape[MAXDIM], out_shape[MAXDIM];
  int64_t lhs_stride[MAXDIM], rhs_stride[MAXDIM], out_stride[MAXDIM];
  int64_t lhs_len, rhs_len, out_len, data_len;
  int real_ndim;
  int64_t real_out_shape[MAXDIM + 1];
} bcast_t;

static void rev(int64_t* a, int n) {
  for (int i = 0; i < n / 2; ++i) { int64_t t = a[i]; a[i] = a[n - 1 - i]; a[n - 1 - i] = t; }
}
static void strides(const int64_t* shape, int n, int64_t* st) {
  if (n == 0) return;
  st[n - 1] = 1;
  for (int i = n - 2; i >= 0; --i) st[i] = st[i + 1] * shape[i + 1];
}
/* lshape/rshape are the FULL shapes (first dim = rows). Returns 0 ok, -1 bad. */
static int calc_bcast(int op, int lnd, const int64_t* lsh, int rnd, const int64_t* rsh, bcast_t* b) {
  memset(b, 0, sizeof(*b));
  int max_ndim = (lnd > rnd ? lnd : rnd) - 1;
  int64_t accum = 0;
  int j = 0, n = 0;
  if (op == O_DOT) {
    b->data_len = lsh[lnd - 1];
    ++j;
    b->real_out_shape[b->real_ndim++] = b->data_len;
  } else {
    b->data_len = 1;
  }
  for (; j < max_ndim; ++j) {
    int64_t dl = (lnd - 1 - j < 1) ? 1 : lsh[lnd - 1 - j];
    int64_t dr = (rnd - 1 - j < 1) ? 1 : rsh[rnd - 1 - j];
    if (dl != dr) {
      if (dl != 1 && dr != 1) return -1;
      if (accum != 0) {
        b->lhs_shape[n] = accum; b->rhs_shape[n] = accum; b->out_shape[n] = accum; ++n;
        accum = 0;
      }
      b->lhs_shape[n] = dl; b->rhs_shape[n] = dr; b->out_shape[n] = dl > dr ? dl : dr; ++n;
    } else {
      accum = accum == 0 ? dl : accum * dl;
    }
    b->real_out_shape[b->real_ndim++] = dl > dr ? dl : dr;
  }
  if (accum != 0) {
    b->lhs_shape[n] = accum; b->rhs_shape[n] = accum; b->out_shape[n] = accum; ++n;
  }
  if (n > MAXDIM) return -1;
  b->ndim = n;
  rev(b->real_out_shape, b->real_ndim);
  rev(b->lhs_shape, n); rev(b->rhs_shape, n); rev(b->out_shape, n);
  strides(b->lhs_shape, n, b->lhs_stride);
  strides(b->rhs_shape, n, b->rhs_stride);
  strides(b->out_shape, n, b->out_stride);
  b->lhs_len = b->rhs_len = b->out_len = 1;
  for (int i = 0; i < n; ++i) {
    b->lhs_len *= b->lhs_shape[i]; b->rhs_len *= b->rhs_shape[i]; b->out_len *= b->out_shape[i];
  }
  return 0;
}
static int has_bcast(int lnd, const int64_t* lsh, int rnd, const int64_t* rsh) {
  if (lnd != rnd) return 1;
  for (int i = 1; i < lnd; ++i) if (lsh[i] != rsh[i]) return 1;
  return 0;
}
/* cpu/binary_reduce_impl.h:56-72 */
static inline int64_t ravel_of(int64_t tx, const bcast_t* b, const int64_t* shape, const int64_t* stride) {
  int64_t out = 0;
  for (int d = 0; d < b->ndim; ++d) {
    int64_t idx = (tx / b->out_stride[d]) % b->out_shape[d];
    int64_t lim = shape[d] - 1;
    out += (idx < lim ? idx : lim) * stride[d];
  }
  return out;
}

/* exported: feature-shape inference (binary_reduce.cc:281-293) */
int ref_infer_binary_feature_shape(const char* op_s, int lnd, const int64_t* lsh, int rnd,
                                   const int64_t* rsh, int64_t* out_shape, int* out_ndim) {
  bcast_t b;
  int op = parse_op(op_s);
  if (op < 0 || calc_bcast(op, lnd, lsh, rnd, rsh, &b)) return -1;
  *out_ndim = b.real_ndim;
  for (int i = 0; i < b.real_ndim; ++i) out_shape[i] = b.real_out_shape[i];
  return 0;
}

typedef struct {
  int64_t num_rows, nnz;
  const int64_t* indptr;
  const int64_t* indices;
  const int64_t* data;
} ref_csr_t;

/*
 * Forward binary reduce.  `csr` is the OUT-CSR (rows = src, cols = dst,
 * data = edge id), traversed like minigun Advance<Config<true,kV2N>>.
 * Maps are nullable; an edge-target map is indexed by out-CSR position and
 * replaces csr.data (cpu/binary_reduce_impl.h:160-169).  `out` is
 * overwritten completely (identity fill first).
 */
int ref_binary_reduce(const char* red_s, const char* op_s, const ref_csr_t* csr,
                      int lhs_tgt, int rhs_tgt,
                      const float* lhs, int lnd, const int64_t* lsh,
                      const float* rhs, int rnd, const int64_t* rsh,
                      float* out, int64_t out_rows, int64_t x_len,
                      const int64_t* lhs_map, const int64_t* rhs_map, const int64_t* out_map,
                      int nthreads) {
  int red = parse_reducer(red_s), op = parse_op(op_s);
  if (red < 0 || op < 0) return -1;
  /* NeedSwitchOrder: binary_reduce.cc:214-219, 318-320 */
  if ((op == O_ADD || op == O_MUL) && lhs_tgt > rhs_tgt) {
    const float* tp = lhs; lhs = rhs; rhs = tp;
    int t = lhs_tgt; lhs_tgt = rhs_tgt; rhs_tgt = t;
    t = lnd; lnd = rnd; rnd = t;
    const int64_t* ts = lsh; lsh = rsh; rsh = ts;
    const int64_t* tm = lhs_map; lhs_map = rhs_map; rhs_map = tm;
  }
  int bc = (op != O_USE_LHS) && has_bcast(lnd, lsh, rnd, rsh);
  bcast_t b;
  int64_t len = 1;
  if (bc) {
    if (calc_bcast(op, lnd, lsh, rnd, rsh, &b)) return -2;
    len = b.data_len;
  } else if (op == O_DOT) {
    len = lsh[lnd - 1];
  }
  const int out_tgt = red == R_NONE ? T_EDGE : T_DST;
  const int64_t* lm = lhs_map ? lhs_map : (lhs_tgt == T_EDGE ? csr->data : NULL);
  const int64_t* rm = rhs_map ? rhs_map : (rhs_tgt == T_EDGE ? csr->data : NULL);
  const int64_t* om = out_map ? out_map : (out_tgt == T_EDGE ? csr->data : NULL);
  const int64_t D = bc ? b.out_len : x_len;
  /* identity fill (single-threaded, cpu/utils.cc:12-17) */
  const float z = red_zero(red);
  for (int64_t i = 0; i < out_rows * D; ++i) out[i] = z;
  const int par = nthreads > 1;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads) if (par)
  for (int64_t r = 0; r < csr->num_rows; ++r) {
    for (int64_t j = csr->indptr[r]; j < csr->indptr[r + 1]; ++j) {
      const int64_t src = r, dst = csr->indices[j], eid = j;
      int64_t lid = sel(lhs_tgt, src, eid, dst);
      int64_t rid = sel(rhs_tgt, src, eid, dst);
      int64_t oid = sel(out_tgt, src, eid, dst);
      if (lm) lid = lm[lid];
      if (rm) rid = rm[rid];
      if (om) oid = om[oid];
      if (!bc) {
        const float* lo = lhs + lid * D * len;
        const float* ro = rhs ? rhs + rid * D * len : NULL;
        float* oo = out + oid * D;
        for (int64_t tx = 0; tx < D; ++tx) {
          float v = op_call(op, lo + tx * len, ro ? ro + tx * len : NULL, len);
          red_call(red, oo + tx, v, par);
        }
      } else {
        const float* lo = lhs + lid * b.lhs_len * len;
        const float* ro = rhs + rid * b.rhs_len * len;
        float* oo = out + oid * b.out_len;
        for (int64_t tx = 0; tx < b.out_len; ++tx) {
          float v = op_call(op, lo + ravel_of(tx, &b, b.lhs_shape, b.lhs_stride) * len,
                            ro + ravel_of(tx, &b, b.rhs_shape, b.rhs_stride) * len, len);
          red_call(red, oo + tx, v, par);
        }
      }
    }
  }
  return 0;
}

/*
 * Backward binary reduce (one side).  `incsr` is the IN-CSR (rows = dst,
 * cols = src, data = edge id); the reference traverses it with src and dst
 * switched (backward_binary_reduce_impl.h:212-245) so the UDF sees the real
 * (src, dst) pair.  Edge-target maps are indexed by in-CSR position.
 * `want` = 0 -> grad_lhs, 1 -> grad_rhs.  The grad buffer is zero-filled and,
 * under broadcasting, has the OUT feature shape (the caller reduces it,
 * tensor.py:572-601).
 */
int ref_backward(const char* red_s, const char* op_s, const ref_csr_t* incsr,
                 int lhs_tgt, int rhs_tgt,
                 const float* lhs, int lnd, const int64_t* lsh,
                 const float* rhs, int rnd, const int64_t* rsh,
                 const float* out, const float* grad_out, int64_t x_len,
                 float* grad, int64_t grad_numel, int want,
                 const int64_t* lhs_map, const int64_t* rhs_map, const int64_t* out_map,
                 int nthreads) {
  int red = parse_reducer(red_s), op = parse_op(op_s);
  if (red < 0 || op < 0) return -1;
  if ((op == O_ADD || op == O_MUL) && lhs_tgt > rhs_tgt) {
    /* BackwardLhs <-> BackwardRhs with swapped operands (binary_reduce.cc:470-476) */
    const float* tp = lhs; lhs = rhs; rhs = tp;
    int t = lhs_tgt; lhs_tgt = rhs_tgt; rhs_tgt = t;
    t = lnd; lnd = rnd; rnd = t;
    const int64_t* ts = lsh; lsh = rsh; rsh = ts;
    const int64_t* tm = lhs_map; lhs_map = rhs_map; rhs_map = tm;
    want = 1 - want;
  }
  int bc = (op != O_USE_LHS) && rhs && has_bcast(lnd, lsh, rnd, rsh);
  bcast_t b;
  int64_t len = 1;
  if (bc) {
    if (calc_bcast(op, lnd, lsh, rnd, rsh, &b)) return -2;
    len = b.data_len;
  } else if (op == O_DOT) {
    len = lsh[lnd - 1];
  }
  const int out_tgt = red == R_NONE ? T_EDGE : T_DST;
  const int64_t* lm = lhs_map ? lhs_map : (lhs_tgt == T_EDGE ? incsr->data : NULL);
  const int64_t* rm = rhs_map ? rhs_map : (rhs_tgt == T_EDGE ? incsr->data : NULL);
  const int64_t* om = out_map ? out_map : (out_tgt == T_EDGE ? incsr->data : NULL);
  for (int64_t i = 0; i < grad_numel; ++i) grad[i] = 0.0f;
  const int par = nthreads > 1;
  if (nthreads < 1) nthreads = 1;
  const int64_t D = bc ? b.out_len : x_len;
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads) if (par)
  for (int64_t r = 0; r < incsr->num_rows; ++r) {
    for (int64_t j = incsr->indptr[r]; j < incsr->indptr[r + 1]; ++j) {
      const int64_t dst = r, src = incsr->indices[j], eid = j;
      int64_t lid = sel(lhs_tgt, src, eid, dst);
      int64_t rid = sel(rhs_tgt, src, eid, dst);
      int64_t oid = sel(out_tgt, src, eid, dst);
      if (lm) lid = lm[lid];
      if (rm) rid = rm[rid];
      if (om) oid = om[oid];
      for (int64_t tx = 0; tx < D; ++tx) {
        const float* lb;
        const float* rb;
        float* gb;
        if (!bc) {
          lb = lhs + lid * D * len + tx * len;
          rb = rhs ? rhs + rid * D * len + tx * len : NULL;
          gb = grad + (want == 0 ? lid : rid) * D * len + tx * len;
        } else {
          lb = lhs + lid * b.lhs_len * len + ravel_of(tx, &b, b.lhs_shape, b.lhs_stride) * len;
          rb = rhs + rid * b.rhs_len * len + ravel_of(tx, &b, b.rhs_shape, b.rhs_stride) * len;
          gb = grad + (want == 0 ? lid : rid) * b.out_len * len + tx * len;
        }
        const float o = out[oid * D + tx];
        const float go = grad_out[oid * D + tx];
        const float e = op_call(op, lb, rb, len);
        const float ge = go * red_bwd(red, e, o);
        for (int64_t i = 0; i < len; ++i) {
          const float l = lb[i];
          const float rr = rb ? rb[i] : 0.0f;
          const float g = want == 0 ? ge * op_bwd_lhs(op, l, rr) : ge * op_bwd_rhs(op, l, rr);
          if (par) {
#pragma omp atomic
            gb[i] += g;
          } else {
            gb[i] += g;
          }
        }
      }
    }
  }
  return 0;
}

/* ---- graph ingestion -------------------------------------------------------- */
/* spmat_op_impl_coo.cc:230-283 (unsorted branch): stable counting sort by row. */
void ref_coo_to_csr(int64_t n_rows, int64_t nnz, const int64_t* row, const int64_t* col,
                    const int64_t* data, int64_t* indptr, int64_t* indices, int64_t* out_data) {
  for (int64_t i = 0; i < n_rows; ++i) indptr[i] = 0;
  for (int64_t i = 0; i < nnz; ++i) indptr[row[i]]++;
  for (int64_t i = 0, c = 0; i < n_rows; ++i) { int64_t t = indptr[i]; indptr[i] = c; c += t; }
  indptr[n_rows] = nnz;
  for (int64_t i = 0; i < nnz; ++i) {
    int64_t r = row[i];
    indices[indptr[r]] = col[i];
    out_data[indptr[r]] = data ? data[i] : i;
    indptr[r]++;
  }
  for (int64_t i = 0, last = 0; i <= n_rows; ++i) { int64_t t = indptr[i]; indptr[i] = last; last = t; }
}

/* spmat_op_impl.cc:323-369 */
void ref_csr_transpose(int64_t n_rows, int64_t n_cols, const int64_t* ap, const int64_t* aj,
                       const int64_t* ax, int64_t* bp, int64_t* bi, int64_t* bx) {
  const int64_t nnz = ap[n_rows];
  for (int64_t i = 0; i < n_cols; ++i) bp[i] = 0;
  for (int64_t j = 0; j < nnz; ++j) bp[aj[j]]++;
  for (int64_t i = 0, c = 0; i < n_cols; ++i) { int64_t t = bp[i]; bp[i] = c; c += t; }
  bp[n_cols] = nnz;
  for (int64_t i = 0; i < n_rows; ++i) {
    for (int64_t j = ap[i]; j < ap[i + 1]; ++j) {
      const int64_t d = aj[j];
      bi[bp[d]] = i;
      bx[bp[d]] = ax ? ax[j] : j;
      bp[d]++;
    }
  }
  for (int64_t i = 0, last = 0; i <= n_cols; ++i) { int64_t t = bp[i]; bp[i] = last; last = t; }
}

/* spmat_op_impl.cc:375-387 */
void ref_csr_to_coo_rows(int64_t n_rows, const int64_t* indptr, int64_t* row) {
  for (int64_t i = 0; i < n_rows; ++i)
    for (int64_t j = indptr[i]; j < indptr[i + 1]; ++j) row[j] = i;
}

int ref_max_threads(void) { return omp_get_max_threads(); }

/*
 * The reference's copy_u_sum instantiation, specialised the way its template
 * expansion is (CallBinaryReduce<kDLCPU, int32, float, SelectSrc, SelectNone,
 * BinaryUseLhs, ReduceSum>, cpu/binary_reduce_sum.cc:15-23): out-CSR
 * traversal, OpenMP over source rows, `omp atomic` scatter per feature into
 * the destination row, single-threaded zero fill.  Used as the cpu_baseline.
 */
void ref_copy_src_sum_i32(int64_t n_src, const int32_t* indptr, const int32_t* indices,
                          const float* x, float* out, int64_t n_dst, int64_t D, int nthreads) {
  for (int64_t i = 0; i < n_dst * D; ++i) out[i] = 0.0f;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
  for (int64_t r = 0; r < n_src; ++r) {
    const float* xo = x + r * D;
    for (int32_t j = indptr[r]; j < indptr[r + 1]; ++j) {
      float* oo = out + (int64_t)indices[j] * D;
      for (int64_t tx = 0; tx < D; ++tx) {
#pragma omp atomic
        oo[tx] += xo[tx];
      }
    }
  }
}
