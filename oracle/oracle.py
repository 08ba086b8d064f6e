"""CPU oracle for the g-SpMM / g-SDDMM path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker.  It wraps
``oracle/build/libdglref.so`` (``dgl_ref.c``, a C restatement of the
reference's CPU kernels) and restates the reference's Python-side glue:

* graph CSR provisioning of a mutable ``DGLGraph``: out-CSR = the adjacency
  lists in edge-id order (``src/graph/graph.cc:600-660``), in-CSR =
  ``CSRTranspose(out-CSR)`` (``src/graph/immutable_graph.cc:407-436``);
* ``BinaryReduce`` / ``CopyReduce`` autograd glue including ``mean`` as
  ``sum / clamp(deg, 1)`` (``python/dgl/backend/pytorch/tensor.py:291-381,
  519-569``) and ``_reduce_grad`` (``tensor.py:572-601``);
* target codes SRC=0 / DST=1 / EDGE=2 / NONE=3 (``function/base.py:7-21``).

Parity status: indexing (COO->CSR, transpose) is pinned bit-exactly by the
reference's literal known-answer arrays (``tests/cpp/test_spmat.cc``, copied
as data into ``tests/golden/spmat_kat.json``); the float arithmetic is pinned
the way the reference's own tests pin it -- differentially against the UDF /
degree-bucketing formulation (``tests/compute/test_kernel.py``), restated in
``oracle/udf_ref.py`` -- plus the closed-form known answers of
``tests/pytorch/test_nn.py``.  The reference library cannot be built or
imported here, so no output of the reference itself exists.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libdglref.so")
_lib = None

SRC, DST, EDGE, NONE = 0, 1, 2, 3


class _CSR(ctypes.Structure):
    _fields_ = [("num_rows", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("indptr", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("data", ctypes.c_void_p)]


def build():
    """Compile the oracle (gcc, OpenMP)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.ref_binary_reduce.restype = ctypes.c_int
        _lib.ref_backward.restype = ctypes.c_int
        _lib.ref_infer_binary_feature_shape.restype = ctypes.c_int
        _lib.ref_max_threads.restype = ctypes.c_int
    return _lib


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _i64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int64)


def _shape(a):
    return (ctypes.c_int64 * len(a.shape))(*a.shape)


# --------------------------------------------------------------------------- #
# Graph ingestion (bit-exact restatements)
# --------------------------------------------------------------------------- #
def coo_to_csr(n_rows, row, col, data=None):
    row, col, data = _i64(row), _i64(col), _i64(data)
    nnz = row.shape[0]
    indptr = np.empty(n_rows + 1, np.int64)
    indices = np.empty(nnz, np.int64)
    out_data = np.empty(nnz, np.int64)
    lib().ref_coo_to_csr(ctypes.c_int64(n_rows), ctypes.c_int64(nnz), _p(row), _p(col),
                         _p(data), _p(indptr), _p(indices), _p(out_data))
    return indptr, indices, out_data


def csr_transpose(n_rows, n_cols, indptr, indices, data=None):
    indptr, indices, data = _i64(indptr), _i64(indices), _i64(data)
    nnz = indices.shape[0]
    bp = np.empty(n_cols + 1, np.int64)
    bi = np.empty(nnz, np.int64)
    bx = np.empty(nnz, np.int64)
    lib().ref_csr_transpose(ctypes.c_int64(n_rows), ctypes.c_int64(n_cols), _p(indptr),
                            _p(indices), _p(data), _p(bp), _p(bi), _p(bx))
    return bp, bi, bx


def csr_to_coo_rows(n_rows, indptr):
    indptr = _i64(indptr)
    row = np.empty(int(indptr[-1]), np.int64)
    lib().ref_csr_to_coo_rows(ctypes.c_int64(n_rows), _p(indptr), _p(row))
    return row


class RefGraph:
    """CSR pair of a mutable DGLGraph built from (src, dst) in edge-id order."""

    def __init__(self, src, dst, num_nodes):
        self.src = _i64(src)
        self.dst = _i64(dst)
        self.n = int(num_nodes)
        self.m = int(self.src.shape[0])
        # out-CSR: adjacency lists keep insertion (eid) order -> stable sort by src
        self.out_csr = coo_to_csr(self.n, self.src, self.dst)
        # in-CSR = transpose of out-CSR: rows ordered by (src asc, eid asc)
        self.in_csr = csr_transpose(self.n, self.n, *self.out_csr)

    def _c(self, csr):
        indptr, indices, data = csr
        c = _CSR(self.n, int(indices.shape[0]), indptr.ctypes.data, indices.ctypes.data,
                 data.ctypes.data)
        c._keep = csr
        return c

    def in_degrees(self):
        return np.diff(self.in_csr[0])

    def out_degrees(self):
        return np.diff(self.out_csr[0])


# --------------------------------------------------------------------------- #
# Kernel-level restatements
# --------------------------------------------------------------------------- #
def infer_binary_feature_shape(op, lhs, rhs):
    out = (ctypes.c_int64 * 9)()
    nd = ctypes.c_int(0)
    rc = lib().ref_infer_binary_feature_shape(op.encode(), lhs.ndim, _shape(lhs), rhs.ndim,
                                              _shape(rhs), out, ctypes.byref(nd))
    if rc != 0:
        raise ValueError("invalid broadcast between %s and %s" % (lhs.shape, rhs.shape))
    return tuple(out[i] for i in range(nd.value))


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def binary_op_reduce_raw(reducer, op, g, lhs_tgt, rhs_tgt, lhs, rhs, out_rows,
                         lhs_map=None, rhs_map=None, out_map=None, nthreads=1):
    """K.binary_op_reduce: fills and returns `out` (no mean division)."""
    lhs, rhs = _f32(lhs), _f32(rhs)
    if rhs is None:
        rhs_shape = lhs.shape
        feat = tuple(lhs.shape[1:])
        out_feat = feat
    else:
        rhs_shape = rhs.shape
        feat = infer_binary_feature_shape(op, lhs, rhs)
        out_feat = feat[:-1] if op == "dot" else feat
    out = np.empty((out_rows,) + tuple(out_feat), np.float32)
    x_len = int(np.prod(out_feat)) if len(out_feat) else 1
    c = g._c(g.out_csr)
    rs = (ctypes.c_int64 * len(rhs_shape))(*rhs_shape)
    lm, rm, om = _i64(lhs_map), _i64(rhs_map), _i64(out_map)
    rc = lib().ref_binary_reduce(
        reducer.encode(), op.encode(), ctypes.byref(c), lhs_tgt, rhs_tgt,
        _p(lhs), lhs.ndim, _shape(lhs), _p(rhs), len(rhs_shape), rs,
        _p(out), ctypes.c_int64(out_rows), ctypes.c_int64(x_len),
        _p(lm), _p(rm), _p(om), nthreads)
    if rc != 0:
        raise ValueError("ref_binary_reduce failed (%d)" % rc)
    return out


def backward_raw(reducer, op, g, lhs_tgt, rhs_tgt, lhs, rhs, out, grad_out, want,
                 lhs_map=None, rhs_map=None, out_map=None, nthreads=1):
    """K.backward_{lhs,rhs}_binary_op_reduce: returns the (un-reduced) grad."""
    lhs, rhs, out, grad_out = _f32(lhs), _f32(rhs), _f32(out), _f32(grad_out)
    if rhs is None:
        feat = tuple(lhs.shape[1:])
        rhs_shape = lhs.shape
    else:
        feat = infer_binary_feature_shape(op, lhs, rhs)
        rhs_shape = rhs.shape
    base = lhs if want == 0 else rhs
    grad = np.empty((base.shape[0],) + tuple(feat), np.float32)
    x_len = int(np.prod(out.shape[1:])) if out.ndim > 1 else 1
    c = g._c(g.in_csr)
    rs = (ctypes.c_int64 * len(rhs_shape))(*rhs_shape)
    lm, rm, om = _i64(lhs_map), _i64(rhs_map), _i64(out_map)
    rc = lib().ref_backward(
        reducer.encode(), op.encode(), ctypes.byref(c), lhs_tgt, rhs_tgt,
        _p(lhs), lhs.ndim, _shape(lhs), _p(rhs), len(rhs_shape), rs,
        _p(out), _p(grad_out), ctypes.c_int64(x_len), _p(grad), ctypes.c_int64(grad.size),
        want, _p(lm), _p(rm), _p(om), nthreads)
    if rc != 0:
        raise ValueError("ref_backward failed (%d)" % rc)
    return grad


def reduce_grad(grad, shape):
    """tensor.py:572-601: sum the gradient over broadcast dimensions."""
    grad_shape = grad.shape[1:]
    in_shape = tuple(shape[1:])
    if tuple(grad_shape) == in_shape:
        return grad
    num_to_squeeze = len(grad_shape) - len(in_shape)
    in_shape = (1,) * num_to_squeeze + in_shape
    axes = tuple(i + 1 for i, (a, b) in enumerate(zip(grad_shape, in_shape)) if a != b)
    return grad.sum(axis=axes, keepdims=True).reshape(shape)


def _degs(g, target, n_in, out_rows, in_map, out_map):
    ones = np.ones((n_in,), np.float32)
    return binary_op_reduce_raw("sum", "use_lhs", g, target, NONE, ones, None, out_rows,
                                lhs_map=in_map, out_map=out_map)


def binary_reduce(reducer, op, g, lhs_tgt, rhs_tgt, lhs, rhs, out_size, grad_out=None,
                  lhs_map=(None, None), rhs_map=(None, None), out_map=(None, None),
                  nthreads=1):
    """tensor.py:291-381 restated: returns out, and (grad_lhs, grad_rhs) if grad_out given."""
    out = binary_op_reduce_raw("sum" if reducer == "mean" else reducer, op, g, lhs_tgt,
                               rhs_tgt, lhs, rhs, out_size, lhs_map[0], rhs_map[0],
                               out_map[0], nthreads)
    degs = None
    if reducer == "mean":
        if lhs_tgt != DST:
            target, n, in_map = lhs_tgt, lhs.shape[0], lhs_map[0]
        else:
            target, n, in_map = rhs_tgt, rhs.shape[0], rhs_map[0]
        degs = _degs(g, target, n, out_size, in_map, out_map[0])
        degs = np.maximum(degs.reshape((out_size,) + (1,) * (out.ndim - 1)), 1)
        out = (out / degs).astype(np.float32)
    if grad_out is None:
        return out
    go = grad_out / degs if degs is not None else grad_out
    red = "sum" if reducer == "mean" else reducer
    gl = backward_raw(red, op, g, lhs_tgt, rhs_tgt, lhs, rhs, out, go, 0,
                      lhs_map[1], rhs_map[1], out_map[1], nthreads)
    gr = backward_raw(red, op, g, lhs_tgt, rhs_tgt, lhs, rhs, out, go, 1,
                      lhs_map[1], rhs_map[1], out_map[1], nthreads)
    return out, reduce_grad(gl, lhs.shape), reduce_grad(gr, rhs.shape)


def copy_reduce(reducer, g, target, x, out_size, grad_out=None, in_map=(None, None),
                out_map=(None, None), nthreads=1):
    """tensor.py:519-569 restated."""
    out = binary_op_reduce_raw("sum" if reducer == "mean" else reducer, "use_lhs", g, target,
                               NONE, x, None, out_size, in_map[0], None, out_map[0], nthreads)
    degs = None
    if reducer == "mean":
        degs = _degs(g, target, x.shape[0], out_size, in_map[0], out_map[0])
        degs = np.maximum(degs.reshape((out_size,) + (1,) * (out.ndim - 1)), 1)
        out = (out / degs).astype(np.float32)
    if grad_out is None:
        return out
    go = grad_out / degs if degs is not None else grad_out
    gx = backward_raw("sum" if reducer == "mean" else reducer, "use_lhs", g, target, NONE,
                      x, None, out, go, 0, in_map[1], None, out_map[1], nthreads)
    return out, gx


def copy_src_sum_i32(n_src, indptr, indices, x, n_dst, nthreads):
    """The reference's specialised copy_u_sum on the out-CSR (cpu_baseline)."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty((n_dst,) + x.shape[1:], np.float32)
    D = int(np.prod(x.shape[1:]))
    lib().ref_copy_src_sum_i32(ctypes.c_int64(n_src), _p(indptr), _p(indices), _p(x), _p(out),
                               ctypes.c_int64(n_dst), ctypes.c_int64(D), nthreads)
    return out


def max_threads():
    return lib().ref_max_threads()


def edge_softmax(g, score):
    """python/dgl/nn/pytorch/softmax.py:33-78 restated on the kernels above:
    copy_e max -> e_sub_v -> exp -> copy_e sum -> e_div_v (no fusion)."""
    score = _f32(score)
    smax = copy_reduce("max", g, EDGE, score, g.n)
    out = binary_op_reduce_raw("none", "sub", g, EDGE, DST, score, smax, g.m)
    with np.errstate(invalid="ignore", over="ignore"):
        out = np.exp(out).astype(np.float32)
    out_sum = copy_reduce("sum", g, EDGE, out, g.n)
    with np.errstate(invalid="ignore", divide="ignore"):
        return binary_op_reduce_raw("none", "div", g, EDGE, DST, out, out_sum, g.m)


# --------------------------------------------------------------------------- #
# The hack's GPU-only entry points (oracle/hack_ref.c)
# --------------------------------------------------------------------------- #
def _f32c(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def csr_sorted_by_edge_type(src, dst, etypes, num_nodes, num_types, transpose):
    """``Graph::GetCsrSortedByEdgeType`` (``src/graph/graph.cc:690-746``): the
    adjacency lists of a mutable graph (insertion = edge-id order per node) with every
    row's entries ordered by edge type.  transpose=False: in-edges (rows = destinations,
    ids = sources); True: out-edges (rows = sources, ids = destinations)."""
    rows, ids = (_i64(src), _i64(dst)) if transpose else (_i64(dst), _i64(src))
    indptr, cols, eids = coo_to_csr(num_nodes, rows, ids)
    et = _i64(etypes)
    o_ids, o_eids, o_types = (np.empty_like(cols) for _ in range(3))
    rc = lib().hack_sort_rows_by_type(ctypes.c_int64(num_nodes), _p(indptr), _p(cols), _p(eids),
                                      _p(et), ctypes.c_int64(num_types), _p(o_ids), _p(o_eids),
                                      _p(o_types))
    if rc != 0:
        raise ValueError("edge type out of range")
    return indptr, o_ids, o_eids, o_types


def hack_fused_gat(src, dst, num_nodes, feat_src, el, er, slope):
    """``FusedGatKernelImpl`` (``binary_reduce_impl.cu:47-112``) on the in-CSR of the
    graph's immutable index (``CSRTranspose`` of the out-CSR, as ``get_immutable_gidx``
    builds it).  Returns (exp (E,H), sum (N,H), ret (N,H,D))."""
    g = RefGraph(src, dst, num_nodes)
    fs, el, er = _f32c(feat_src), _f32c(el), _f32c(er)
    n, H, D = fs.shape[0], el.reshape(el.shape[0], -1).shape[1], fs.shape[-1]
    indptr, indices, data = g.in_csr
    exp = np.empty((g.m, H), np.float32)
    s = np.empty((n, H), np.float32)
    ret = np.empty((n, H, D), np.float32)
    lib().hack_fused_gat(ctypes.c_int64(n), _p(indptr), _p(indices), _p(data), ctypes.c_int64(H),
                         ctypes.c_int64(D), _p(fs), _p(el), _p(er), ctypes.c_float(slope), _p(exp),
                         _p(s), _p(ret))
    return exp, s, ret


def hack_fused_gat_backward(src, dst, num_nodes, feat_src, el, er, s, exp, ret, grad_out, slope):
    """``BackwardFusedGatKernelImpl`` (``binary_reduce_impl.cu:1248-1308``) on the
    out-CSR.  Returns (grad_feat_src, grad_el, grad_er)."""
    g = RefGraph(src, dst, num_nodes)
    fs, el, er = _f32c(feat_src), _f32c(el), _f32c(er)
    s, exp, ret, go = _f32c(s), _f32c(exp), _f32c(ret), _f32c(grad_out)
    n, H, D = fs.shape[0], s.shape[1], fs.shape[-1]
    indptr, indices, data = g.out_csr
    gfs = np.empty_like(fs)
    gel = np.zeros((n, H), np.float32)
    ger = np.zeros((n, H), np.float32)
    lib().hack_fused_gat_backward(ctypes.c_int64(n), _p(indptr), _p(indices), _p(data),
                                  ctypes.c_int64(H), ctypes.c_int64(D), _p(fs), _p(el), _p(er),
                                  _p(s), _p(exp), _p(ret), _p(go), ctypes.c_float(slope), _p(gfs),
                                  _p(gel), _p(ger))
    return gfs, gel.reshape(el.shape), ger.reshape(er.shape)


def hack_rgcn_layer0(src, dst, etypes, num_nodes, weight, norm):
    """``RgcnLayer0Impl`` (``binary_reduce_impl.cu:913-980``): weight (R, N, F)."""
    w, nm = _f32c(weight), _f32c(norm).reshape(-1)
    R, F = w.shape[0], w.shape[2]
    ranges, ids, eids, types = csr_sorted_by_edge_type(src, dst, etypes, num_nodes, R, False)
    ret = np.empty((num_nodes, F), np.float32)
    lib().hack_rgcn_layer0(ctypes.c_int64(num_nodes), _p(ranges), _p(ids), _p(eids), _p(types),
                           _p(w), ctypes.c_int64(w.shape[1]), ctypes.c_int64(F), _p(nm), _p(ret))
    return ret


def hack_rgcn_layer0_backward(src, dst, etypes, num_nodes, grad_out, norm, num_rels,
                              accumulate=True):
    """``RgcnLayer0BackwardImpl`` (``:982-1047``); ``accumulate=False`` keeps the
    reference's store (repeated (source, relation) pairs keep the last edge)."""
    go, nm = _f32c(grad_out), _f32c(norm).reshape(-1)
    F = go.shape[1]
    ranges, ids, eids, types = csr_sorted_by_edge_type(src, dst, etypes, num_nodes, num_rels, True)
    gw = np.zeros((num_rels, num_nodes, F), np.float32)
    lib().hack_rgcn_layer0_backward(ctypes.c_int64(num_nodes), _p(ranges), _p(ids), _p(eids),
                                    _p(types), _p(go), _p(nm), ctypes.c_int64(F),
                                    ctypes.c_int(1 if accumulate else 0), _p(gw))
    return gw


def hack_rgcn_layer1(src, dst, etypes, num_nodes, hidden, weight, norm):
    """``RgcnLayer1Impl`` (``:1082-1155``): hidden (N, Y), weight (R, Y, X)."""
    h, w, nm = _f32c(hidden), _f32c(weight), _f32c(norm).reshape(-1)
    R, Y, X = w.shape
    ranges, ids, eids, types = csr_sorted_by_edge_type(src, dst, etypes, num_nodes, R, False)
    ret = np.zeros((num_nodes, X), np.float32)
    lib().hack_rgcn_layer1(ctypes.c_int64(num_nodes), _p(ranges), _p(ids), _p(eids), _p(types),
                           _p(h), _p(w), ctypes.c_int64(Y), ctypes.c_int64(X), _p(nm), _p(ret))
    return ret


def hack_rgcn_layer1_backward(src, dst, etypes, num_nodes, hidden, weight, norm, grad_out):
    """``RgcnLayer1BackwardImpl`` (``:1157-1245``).  Returns (grad_hidden, grad_weight)."""
    h, w, nm, go = _f32c(hidden), _f32c(weight), _f32c(norm).reshape(-1), _f32c(grad_out)
    R, Y, X = w.shape
    ranges, ids, eids, types = csr_sorted_by_edge_type(src, dst, etypes, num_nodes, R, True)
    gh = np.zeros((num_nodes, Y), np.float32)
    gw = np.zeros((R, Y, X), np.float32)
    lib().hack_rgcn_layer1_backward(ctypes.c_int64(num_nodes), _p(ranges), _p(ids), _p(eids),
                                    _p(types), _p(h), _p(w), ctypes.c_int64(Y), ctypes.c_int64(X),
                                    _p(nm), _p(go), _p(gh), _p(gw))
    return gh, gw
