"""Backend operator layer: autograd Functions over the kernels.

Mirrors the reference's operator contract ``F.binary_reduce`` /
``F.copy_reduce`` (``python/dgl/backend/backend.py:1189-1225, 1276-1302``)
and its PyTorch implementation (``backend/pytorch/tensor.py:291-381,
519-601``):

* the output is allocated by the operator (``new_empty``) and filled by the
  kernel;
* ``mean`` is ``sum`` divided by ``clamp(deg, 1)``, where the degree is a
  second ``copy_reduce('sum')`` over ones (``tensor.py:308-325, 530-539``);
* gradients of broadcast operands are summed over the broadcast dimensions
  (``_reduce_grad``, ``tensor.py:572-601``);
* mappings are ``(forward, backward)`` pairs; node maps are node-id
  indexed, and in this engine edge maps are edge-id indexed (see
  include/dglmi.h), so both entries of an edge pair are usually the same.
"""
from __future__ import annotations

import os
import weakref

import torch as th

from . import kernel as K
from ._ffi import DGLError

SRC, DST, EDGE, NONE = 0, 1, 2, 3
_NOMAP = (None, None)


def _degs(reducer_target, graph, n, out_size, in_map, out_map, like):
    """In-degrees for ``mean`` (tensor.py:308-325 counts them with a copy_reduce of
    ones each call).  Unmapped calls read the cached CSR degrees instead -- the
    integers (exact in fp32 below 2^24, where a sum of ones stops counting)."""
    if in_map is None and out_map is None and out_size == graph.in_csr.num_rows:
        return graph.in_csr.degrees().to(like.dtype)
    ones = like.new_ones((n,))
    degs = like.new_empty((out_size,))
    K.copy_reduce("sum", graph, reducer_target, ones, degs, in_map, out_map)
    return degs


class BinaryReduce(th.autograd.Function):
    @staticmethod
    def forward(ctx, reducer, binary_op, graph, lhs, rhs, lhs_data, rhs_data, out_data,
                out_size, lhs_map, rhs_map, out_map):
        feat_shape = K.infer_binary_feature_shape(binary_op, lhs_data, rhs_data)
        degs = None
        if reducer == "mean":
            if lhs != DST:
                target, n, in_map = lhs, lhs_data.shape[0], lhs_map[0]
            else:
                target, n, in_map = rhs, rhs_data.shape[0], rhs_map[0]
            degs = _degs(target, graph, n, out_data.shape[0], in_map, out_map[0], lhs_data)
            degs = degs.clamp(min=1)
        # mean = the sum divided by the in-degree in the kernel's epilogue (one pass)
        K.binary_op_reduce(reducer if reducer != "mean" else "sum", binary_op, graph, lhs, rhs,
                           lhs_data, rhs_data, out_data, lhs_map[0], rhs_map[0], out_map[0],
                           epilogue=None if degs is None else (None, degs, None))
        if degs is not None:
            degs = degs.reshape((out_data.shape[0],) + (1,) * (out_data.dim() - 1))
        ctx.backward_cache = (reducer, binary_op, graph, lhs, rhs, lhs_map, rhs_map, out_map,
                              feat_shape, degs)
        ctx.save_for_backward(lhs_data, rhs_data, out_data)
        return out_data

    @staticmethod
    def backward(ctx, grad_out):
        (reducer, binary_op, graph, lhs, rhs, lhs_map, rhs_map, out_map, feat_shape,
         degs) = ctx.backward_cache
        lhs_data, rhs_data, out_data = ctx.saved_tensors
        grad_lhs = grad_rhs = None
        if reducer == "mean":
            grad_out = grad_out / degs
        grad_out = grad_out.contiguous()
        red = reducer if reducer != "mean" else "sum"
        fused = _edge_grad_by_dot(red, binary_op, graph, lhs, rhs, lhs_data, rhs_data, grad_out,
                                  lhs_map, rhs_map, out_map, ctx.needs_input_grad[5],
                                  ctx.needs_input_grad[6])
        if fused is not None:
            return (None, None, None, None, None) + fused + (None,) * 5
        if ctx.needs_input_grad[5]:
            grad_lhs = grad_out.new_empty((lhs_data.shape[0],) + tuple(feat_shape))
            K.backward_lhs_binary_op_reduce(red, binary_op, graph, lhs, rhs, lhs_data, rhs_data,
                                            out_data, grad_out, grad_lhs, lhs_map[1], rhs_map[1],
                                            out_map[1])
            grad_lhs = _reduce_grad(grad_lhs, lhs_data.shape)
        if ctx.needs_input_grad[6]:
            grad_rhs = grad_out.new_empty((rhs_data.shape[0],) + tuple(feat_shape))
            K.backward_rhs_binary_op_reduce(red, binary_op, graph, lhs, rhs, lhs_data, rhs_data,
                                            out_data, grad_out, grad_rhs, lhs_map[1], rhs_map[1],
                                            out_map[1])
            grad_rhs = _reduce_grad(grad_rhs, rhs_data.shape)
        return None, None, None, None, None, grad_lhs, grad_rhs, None, None, None, None, None


def _edge_grad_by_dot(red, op, graph, lhs, rhs, lhs_data, rhs_data, grad_out, lhs_map, rhs_map,
                      out_map, need_l, need_r):
    """u_mul_e_sum with the edge operand broadcast over the last feature dim
    (GAT: ft (N, H, D) x a (E, H, 1)).  The reference materialises the edge
    gradient in the broadcast OUTPUT shape (E, H, D) and sums it afterwards
    (tensor.py:350-356, 572-601) -- E*H*D floats written and re-read.  The same
    numbers come from one SDDMM: grad_a[e, h] = sum_d grad_out[dst, h, d] *
    ft[src, h, d] = u_dot_v(ft, grad_out), so the edge gradient is computed
    directly in its own shape.  The node gradient is the regular kernel."""
    if op != "mul" or red != "sum":
        return None
    if any(m is not None for pair in (lhs_map, rhs_map, out_map) for m in pair):
        return None
    if not (need_l or need_r):
        return None
    if lhs == SRC and rhs == EDGE:
        node, edge, node_first = lhs_data, rhs_data, True
    elif lhs == EDGE and rhs == SRC:
        node, edge, node_first = rhs_data, lhs_data, False
    else:
        return None
    if node.dim() != edge.dim() or node.dim() < 2 or edge.shape[-1] != 1 or node.shape[-1] == 1 \
            or tuple(edge.shape[1:-1]) != tuple(node.shape[1:-1]):
        return None
    need_edge = need_r if node_first else need_l
    g_edge = None
    if need_edge:  # (skipped for constant edge weights, e.g. R-GCN norms)
        g_edge = grad_out.new_empty((edge.shape[0],) + tuple(node.shape[1:-1]))
        K.binary_op_reduce("none", "dot", graph, SRC, DST, node, grad_out, g_edge)
        g_edge = g_edge.view(edge.shape)
    g_node = None
    need_node = need_l if node_first else need_r
    if need_node:
        g_node = grad_out.new_empty(node.shape)
        if node_first:
            K.backward_lhs_binary_op_reduce("sum", "mul", graph, lhs, rhs, lhs_data, rhs_data,
                                            grad_out, grad_out, g_node)
        else:
            K.backward_rhs_binary_op_reduce("sum", "mul", graph, lhs, rhs, lhs_data, rhs_data,
                                            grad_out, grad_out, g_node)
    return (g_node, g_edge) if node_first else (g_edge, g_node)


def binary_reduce(reducer, binary_op, graph, lhs, rhs, lhs_data, rhs_data, out_size,
                  lhs_map=_NOMAP, rhs_map=_NOMAP, out_map=_NOMAP):
    """backend.py:1189-1225 / tensor.py:368-381."""
    lhs_data = lhs_data.contiguous()
    rhs_data = rhs_data.contiguous()
    feat_shape = K.infer_binary_feature_shape(binary_op, lhs_data, rhs_data)
    out_shape = feat_shape[:-1] if binary_op == "dot" else feat_shape
    out_data = lhs_data.new_empty((out_size,) + tuple(out_shape))
    if _streams_edge_operand(reducer, binary_op, graph, lhs, rhs, lhs_data, rhs_data, out_size,
                             lhs_map, rhs_map, out_map):
        return _StreamedEdgeReduce.apply(reducer, binary_op, graph, lhs, rhs, lhs_data, rhs_data,
                                         out_data)
    return BinaryReduce.apply(reducer, binary_op, graph, lhs, rhs, lhs_data, rhs_data, out_data,
                              out_size, lhs_map, rhs_map, out_map)


# edges from which a constant edge operand is streamed in walk order (below), and the
# widest per-edge operand (floats) worth a cached permuted copy
STREAM_EDGE_MIN_EDGES = 1 << 20
STREAM_EDGE_MAX_WIDTH = 8


def _streams_edge_operand(reducer, op, graph, lhs, rhs, lhs_data, rhs_data, out_size, lhs_map,
                          rhs_map, out_map):
    """True for u_op_e / e_op_u reductions to destinations whose edge operand needs no
    gradient (R-GCN / GCN edge norms, fixed edge weights) on a large graph: the kernels
    read such an operand by edge id, one random line per edge once it outgrows the
    caches (C5 graph: u_mul_e_sum 5.55 ms against copy_u_sum's 3.47 ms), so it is
    streamed in the walk's position order instead (ImmutableGraphIndex.position_operand:
    a permuted copy, built once per direction and cached while the tensor and its
    version counter are unchanged).  Narrow operands only: the copy costs its size;
    and only from an operand's second use on (a tensor made fresh every call, such as
    an attention computed without grad, keeps the edge-id walk: permuting it each
    call cost the C3 unfused GAT forward 21 -> 44 ms)."""
    if reducer not in ("sum", "mean", "max", "min") or op == "dot":
        return False
    if sorted((lhs, rhs)) != [SRC, EDGE]:
        return False
    if any(m is not None for pair in (lhs_map, rhs_map, out_map) for m in pair):
        return False
    edge = rhs_data if rhs == EDGE else lhs_data
    if edge.requires_grad or not edge.is_cuda or os.environ.get("DGLMI_STREAM_EDGE", "1") == "0":
        return False
    # whole graphs only (edge ids a permutation of [0, nnz)), not a position view, and
    # not a graph whose in-CSR already holds its edges in id order (read at the position)
    if not getattr(graph, "eid_perm", False) or getattr(graph, "position_of", None) is not None:
        return False
    if graph.eid_identity_bits() & 1:
        return False
    ic = graph.in_csr
    return (ic.nnz >= STREAM_EDGE_MIN_EDGES and edge.shape[0] == ic.nnz
            and out_size == ic.num_rows and edge[0].numel() <= STREAM_EDGE_MAX_WIDTH
            and graph.reused_operand(edge))


class _StreamedEdgeReduce(th.autograd.Function):
    """BinaryReduce with the constant edge operand in walk order: the forward walks
    the in-CSR view whose edge ids are its positions (the operand permuted to match),
    the node gradient walks the out-CSR view with the operand in out-CSR order.
    Bit-identical to the edge-id walk (the same values in the same summation order)."""

    @staticmethod
    def forward(ctx, reducer, op, graph, lhs, rhs, lhs_data, rhs_data, out_data):
        edge_is_rhs = rhs == EDGE
        vin, e_in = graph.position_operand(rhs_data if edge_is_rhs else lhs_data, "in")
        l_in, r_in = (lhs_data, e_in) if edge_is_rhs else (e_in, rhs_data)
        degs = None
        if reducer == "mean":
            degs = graph.in_csr.degrees().to(lhs_data.dtype).clamp(min=1)
        K.binary_op_reduce(reducer if reducer != "mean" else "sum", op, vin, lhs, rhs, l_in,
                           r_in, out_data, epilogue=None if degs is None else (None, degs, None))
        if degs is not None:
            degs = degs.reshape((out_data.shape[0],) + (1,) * (out_data.dim() - 1))
        ctx.cache = (reducer, op, graph, lhs, rhs, edge_is_rhs, degs)
        ctx.save_for_backward(lhs_data, rhs_data, out_data)
        return out_data

    @staticmethod
    def backward(ctx, grad_out):
        reducer, op, graph, lhs, rhs, edge_is_rhs, degs = ctx.cache
        lhs_data, rhs_data, out_data = ctx.saved_tensors
        node_idx = 5 if edge_is_rhs else 6
        if not ctx.needs_input_grad[node_idx]:
            return (None,) * 8
        if degs is not None:
            grad_out = grad_out / degs
        grad_out = grad_out.contiguous()
        red = reducer if reducer != "mean" else "sum"
        vout, e_out = graph.position_operand(rhs_data if edge_is_rhs else lhs_data, "out")
        feat_shape = K.infer_binary_feature_shape(op, lhs_data, rhs_data)
        if edge_is_rhs:
            g = grad_out.new_empty((lhs_data.shape[0],) + tuple(feat_shape))
            K.backward_lhs_binary_op_reduce(red, op, vout, lhs, rhs, lhs_data, e_out, out_data,
                                            grad_out, g)
            return None, None, None, None, None, _reduce_grad(g, lhs_data.shape), None, None
        g = grad_out.new_empty((rhs_data.shape[0],) + tuple(feat_shape))
        K.backward_rhs_binary_op_reduce(red, op, vout, lhs, rhs, e_out, rhs_data, out_data,
                                        grad_out, g)
        return None, None, None, None, None, None, _reduce_grad(g, rhs_data.shape), None


class CopyReduce(th.autograd.Function):
    @staticmethod
    def forward(ctx, reducer, graph, target, in_data, out_data, out_size, in_map, out_map):
        degs = None
        if reducer == "mean":
            degs = _degs(target, graph, in_data.shape[0], out_data.shape[0], in_map[0],
                         out_map[0], in_data).clamp(min=1)
        K.copy_reduce(reducer if reducer != "mean" else "sum", graph, target, in_data, out_data,
                      in_map[0], out_map[0],
                      epilogue=None if degs is None else (None, degs, None))
        if degs is not None:
            degs = degs.reshape((out_data.shape[0],) + (1,) * (out_data.dim() - 1))
        ctx.backward_cache = (reducer, graph, target, in_map, out_map, degs)
        ctx.save_for_backward(in_data, out_data)
        return out_data

    @staticmethod
    def backward(ctx, grad_out):
        reducer, graph, target, in_map, out_map, degs = ctx.backward_cache
        in_data, out_data = ctx.saved_tensors
        grad_in = None
        if reducer == "mean":
            grad_out = grad_out / degs
        grad_out = grad_out.contiguous()
        if ctx.needs_input_grad[3]:
            grad_in = grad_out.new_empty(in_data.shape)
            K.backward_copy_reduce(reducer if reducer != "mean" else "sum", graph, target,
                                   in_data, out_data, grad_out, grad_in, in_map[1], out_map[1])
        return None, None, None, grad_in, None, None, None, None


def copy_reduce(reducer, graph, target, in_data, out_size, in_map=_NOMAP, out_map=_NOMAP):
    """backend.py:1276-1302 / tensor.py:566-569."""
    in_data = in_data.contiguous()
    out_data = in_data.new_empty((out_size,) + tuple(in_data.shape[1:]))
    return CopyReduce.apply(reducer, graph, target, in_data, out_data, out_size, in_map, out_map)


def _reduce_grad(grad, shape):
    """tensor.py:572-601: sum the gradient over broadcast dimensions."""
    grad_shape = grad.shape[1:]
    in_shape = tuple(shape[1:])
    if tuple(grad_shape) == in_shape:
        return grad
    num_to_squeeze = len(grad_shape) - len(in_shape)
    in_shape = (1,) * num_to_squeeze + in_shape
    reduce_idx = tuple(i + 1 for i, (a, b) in enumerate(zip(grad_shape, in_shape)) if a != b)
    grad = grad.sum(dim=reduce_idx, keepdim=True)
    return grad.view(shape)


def nb_access_bench(graph, feat, node_map=None, deg_inc_node_map=None, times=15, warm_up_times=5):
    """The hack's neighbour-access microbenchmark (``backend.py:1253``,
    ``tensor.py:422-438``, ``_CAPI_DGLNbAccess`` -> ``binary_reduce_impl.cu:779-...``):
    time the gather of every in-neighbour's feature row over the in-CSR,
    ``times`` launches after ``warm_up_times`` warm-ups, log the average and
    return ``feat`` unchanged.  The reference's kernels read rows without using
    them (the compiler may drop the loads); here the timed launch is the
    load-balanced in-neighbour gather itself (copy_u_sum), whose result is kept
    so the gathers are real.  The node maps of the reference's disabled
    sharding modes are accepted and ignored (``DGLMINbAccess``, the C entry of
    ``_CAPI_DGLNbAccess``).  Returns (feat, average_us)."""
    import sys
    gidx = graph if hasattr(graph, "in_csr") else graph._graph.get_immutable_gidx(feat.device)
    x = feat.contiguous().view(feat.shape[0], -1)
    avg = K.nb_access(gidx, x, node_map, deg_inc_node_map, times, warm_up_times)
    print("feat_len:%d num_nodes:%d num_edges:%d -- neighbour gather takes %.1f us on average"
          % (x.shape[1], gidx.in_csr.num_rows, gidx.in_csr.nnz, avg), file=sys.stderr)
    return feat, avg


# --------------------------------------------------------------------------- #
# dense projections that bracket the aggregations (MFMA GEMMs)
# --------------------------------------------------------------------------- #
def weight_grad(x, gy):
    """dW = X^T dY for a feature projection Y = X W over N nodes (N >> F).

    As one GEMM the whole node dimension is the reduction: a (F_in x F_out)
    output of a few hundred tiles cannot fill 256 CUs and hipBLASLt runs it at
    1-2 TB/s (5.6 ms for N = 5 M, 64 -> 256).  Split-K instead: the node rows are
    cut into S slices, one batched GEMM computes the S partial products on MFMA
    (S x more tiles) and a sum folds them (1.35 ms; 0.41 -> 0.07 ms at the arxiv
    shape; scripts/gemm_splitk_probe.py)."""
    k, n = x.shape[-1], gy.shape[-1]
    x2 = x.reshape(-1, k).contiguous()
    g2 = gy.reshape(-1, n).contiguous()
    m = x2.shape[0]
    s = 1
    while s * 2 <= min(128, m // 1024):
        s *= 2
    if s < 8:
        return x2.t() @ g2
    mm = (m // s) * s
    out = th.bmm(x2[:mm].view(s, mm // s, k).transpose(1, 2), g2[:mm].view(s, mm // s, n)).sum(0)
    if mm < m:
        out.addmm_(x2[mm:].t(), g2[mm:])
    return out


class _Project(th.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        x2 = x.reshape(-1, x.shape[-1])
        if K.project_mfma_ok(x2, w) and (b is None or K.project_bias_ok(b, w.shape[1], x2.device)):
            # tall-skinny: the MFMA kernel with W in registers (kernels_project.hip)
            return K.project_mfma(x2, w, b).view(x.shape[:-1] + (w.shape[1],))
        if b is None:
            return th.matmul(x, w)
        # bias in the GEMM epilogue (hipBLASLt addmm), not a separate pass
        return th.addmm(b, x2, w).view(x.shape[:-1] + (w.shape[1],))

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        # a loss like out.sum() hands back an expanded (stride-0) gradient; torch's
        # column sum over such a view took 0.5 ms for 169 343 x 128 (C2 trace)
        # against ~30 us for one dense copy + a dense sum
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gy2 = gy.reshape(-1, gy.shape[-1])
            wt = w.t()
            if K.project_mfma_ok(gy2, wt):
                gx = K.project_mfma(gy2, wt).view(gy.shape[:-1] + (w.shape[0],))
            else:
                gx = th.matmul(gy, wt)
        if ctx.needs_input_grad[1]:
            gw = weight_grad(x, gy)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.reshape(-1, gy.shape[-1]).sum(0)
        return gx, gw, gb


def project(x, w, bias=None):
    """Y = X W (+ bias) (X: (..., F_in), W: (F_in, F_out)) with the split-K weight
    gradient; a bias is added inside the GEMM."""
    if w.dim() != 2:
        y = th.matmul(x, w)
        return y if bias is None else y + bias
    return _Project.apply(x, w, bias)


class _GcnAggregate(th.autograd.Function):
    """out[v] = (sum_{u->v} X[u]) * row_mul[v] / row_div[v] + bias + addend[v] in ONE
    kernel (copy_u_sum with the fused epilogue): GraphConv's aggregation, norm and
    bias (graphconv.py:150-170), the mean reducer's division (tensor.py:308-325) and
    the residual terms of SAGE / GIN / APPNP / Cheb without extra passes over the
    output.  row_mul / row_div are constants (no gradient); addend gets grad_out."""

    @staticmethod
    def forward(ctx, gidx, x, row_mul, bias, n_dst, row_div, addend):
        out = x.new_empty((n_dst, x.shape[1]))
        K.copy_reduce("sum", gidx, SRC, x, out, epilogue=(row_mul, row_div, bias, addend))
        ctx.gidx = gidx
        ctx.save_for_backward(x, out, row_mul, row_div)
        ctx.has_bias = bias is not None
        ctx.has_addend = addend is not None
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, out, row_mul, row_div = ctx.saved_tensors
        gx = gb = ga = None
        g = grad_out.contiguous()
        if ctx.needs_input_grad[1]:
            gs = g
            if row_mul is not None:
                gs = gs * row_mul.view(-1, 1)
            if row_div is not None:
                gs = gs / row_div.view(-1, 1)
            gx = th.empty_like(x)
            K.backward_copy_reduce("sum", ctx.gidx, SRC, x, out, gs.contiguous(), gx)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            gb = g.sum(0)
        if ctx.has_addend and ctx.needs_input_grad[6]:
            ga = g
        return None, gx, None, gb, None, None, ga


def gcn_aggregate(gidx, x, row_mul=None, bias=None, n_dst=None, row_div=None, addend=None):
    """Fused copy_u_sum + epilogue (see _GcnAggregate); x is (N_src, F) float32,
    row_mul / row_div (N_dst,), bias (F,), addend (N_dst, F)."""
    n_dst = gidx.in_csr.num_rows if n_dst is None else n_dst
    if addend is not None:
        addend = addend.contiguous()
    return _GcnAggregate.apply(gidx, x.contiguous(), row_mul, bias, n_dst, row_div, addend)


class _GcnNormAggregate(th.autograd.Function):
    """GraphConv's normalised aggregation with BOTH norms folded into one constant
    per-edge weight w_e (``ImmutableGraphIndex.gcn_edge_weights``, streamed in walk
    order): out[v] = sum_{u->v} w_e X[u] + bias in one launch, and the gradient
    dX[u] = sum_{u->v} w_e dOut[v] in one out-CSR launch -- no elementwise passes
    for the source-side scaling of X, its gradient, or the destination-side scaling
    of the incoming gradient (three (N, F) read + write passes per layer)."""

    @staticmethod
    def forward(ctx, gidx, x, norm, bias, n_dst):
        vin, w_in, _, _ = gidx.gcn_edge_weights(norm)
        out = x.new_empty((n_dst, x.shape[1]))
        epi = None if bias is None else (None, None, bias, None)
        K.binary_op_reduce("sum", "mul", vin, SRC, EDGE, x, w_in, out, epilogue=epi)
        ctx.gidx, ctx.norm, ctx.has_bias = gidx, norm, bias is not None
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, out = ctx.saved_tensors
        g = grad_out.contiguous()
        gx = gb = None
        if ctx.needs_input_grad[1]:
            _, _, vout, w_out = ctx.gidx.gcn_edge_weights(ctx.norm)
            gx = th.empty_like(x)
            K.backward_lhs_binary_op_reduce("sum", "mul", vout, SRC, EDGE, x, w_out, out, g, gx)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            gb = g.sum(0)
        return None, gx, None, gb, None


def gcn_norm_aggregate(gidx, x, norm, bias=None, n_dst=None):
    """GraphConv aggregation of the UNnormalised features ``x`` (N_src, F) with
    norm ``"both"`` or ``"right"`` applied through per-edge weights (see
    _GcnNormAggregate).  Needs a whole graph (edge ids a permutation)."""
    if norm not in ("both", "right"):
        raise DGLError("gcn_norm_aggregate: norm must be 'both' or 'right'")
    n_dst = gidx.in_csr.num_rows if n_dst is None else n_dst
    return _GcnNormAggregate.apply(gidx, x.contiguous(), norm, bias, n_dst)


# where the fused walks read the caller's dropout mask: "<forward>,<backward>", each "eid"
# (a random word per edge, in the walk) or "pos" (gathered into walk order first)
GAT_KEEP_ORDER = "pos,pos"


class FusedGat(th.autograd.Function):
    """tensor.py:383-413 (FusedGat), max-stabilised and without per-edge buffers.  When
    a gradient will be wanted, the forward also keeps the attention's slope aggregates
    (DGLMIFusedGatForwardEx: N x H x D + N x H floats), and the backward is a dense pass
    plus the source-side walk -- no destination-side walk.
    DGLMI_GAT_SLOPES=0 keeps the round-3 backward (destination walk / edge positions).
    ``attn_drop`` > 0: GATConv's attention dropout (gatconv.py:154) inside the same
    kernels, the mask a hash of ``seed`` and the edge id, recomputed by the backward
    (DGLMIFusedGatDropout*; always with the slope aggregates).  ``keep`` (E,) keep
    words with ``keep_scale`` instead: the caller's mask (DGLMIFusedGatKeep*; GATConv's
    own nn.Dropout draws).  ``draw`` (dgl.kernel.dropout_draw) instead: torch's own draws
    recomputed inside the walks (DGLMIFusedGatDraw*; no mask in memory)."""

    @staticmethod
    def forward(ctx, gidx, feat_src, el, er, slope, attn_drop=0.0, seed=0, keep=None,
                keep_scale=None, draw=None):
        feat_src, el, er = feat_src.contiguous(), el.contiguous(), er.contiguous()
        n_dst = er.shape[0]
        H, D = feat_src.shape[1], feat_src.shape[2]
        out = feat_src.new_empty((n_dst, H, D))
        mx = feat_src.new_empty((n_dst, H))
        sm = feat_src.new_empty((n_dst, H))
        lf = ls = None
        if any(ctx.needs_input_grad[1:4]) and (
                attn_drop > 0.0 or keep is not None or draw is not None
                or os.environ.get("DGLMI_GAT_SLOPES", "1") != "0"):
            lf = feat_src.new_empty((n_dst, H, D))
            ls = feat_src.new_empty((n_dst, H))
        keep_in = keep_out = None
        # the caller's mask per direction: by edge id (the walk reads a random word per
        # edge) or gathered into the walk's position order first (DGLMIGatKeepGather: the
        # same random reads in a pass of their own, then coalesced reads in the walk);
        # DGLMI_GAT_KEEP_ORDER = "<fwd>,<bwd>" with each "eid" or "pos" (A/B)
        order = os.environ.get("DGLMI_GAT_KEEP_ORDER", GAT_KEEP_ORDER).split(",")
        pos_in, pos_out = order[0] == "pos", order[-1] == "pos"
        if keep is not None:
            keep_in = K.gat_keep_walk_order(gidx, keep, feat_src, "in") if pos_in else keep
            if lf is not None:
                keep_out = K.gat_keep_walk_order(gidx, keep, feat_src, "out") if pos_out else keep
        K.fused_gat_forward(gidx, feat_src, el, er, slope, out, mx, sm, lf, ls,
                            attn_drop=attn_drop, seed=seed, keep=keep_in, keep_scale=keep_scale,
                            keep_pos=pos_in, draw=draw)
        del keep_in
        ctx.draw = draw
        ctx.gidx, ctx.slope = gidx, slope
        ctx.attn_drop, ctx.seed = attn_drop, seed
        ctx.keep, ctx.keep_scale, ctx.keep_pos = keep_out, keep_scale, pos_out
        ctx.slopes = lf is not None
        if lf is not None:
            ctx.save_for_backward(feat_src, el, er, out, mx, sm, lf, ls)
        else:
            ctx.save_for_backward(feat_src, el, er, out, mx, sm)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        saved = ctx.saved_tensors
        feat_src, el, er, out, mx, sm = saved[:6]
        lf, ls = saved[6:] if ctx.slopes else (None, None)
        grad_out = grad_out.contiguous()
        g_ft = th.empty_like(feat_src)
        g_el = th.empty_like(el)
        g_er = th.empty_like(er)
        K.fused_gat_backward(ctx.gidx, feat_src, el, er, ctx.slope, out, mx, sm, grad_out, g_ft,
                             g_el, g_er, lf, ls, attn_drop=ctx.attn_drop, seed=ctx.seed,
                             keep=ctx.keep, keep_scale=ctx.keep_scale,
                             keep_pos=getattr(ctx, "keep_pos", False), draw=ctx.draw)
        return None, g_ft, g_el, g_er, None, None, None, None, None, None


def fused_gat(graph, feat_src, el, er, slope, attn_drop=0.0, seed=None, keep=None,
              keep_scale=None, draw=None):
    """backend.py:1235 / tensor.py:415-420: softmax attention + aggregation in one kernel.

    ``graph`` is a DGLGraph (or an ImmutableGraphIndex); feat_src (N, H, D), el / er
    (N, H, 1).  Returns (N, H, D).  Attention dropout, two forms:

    * ``keep`` (E,) keep words in edge-id order (:func:`dgl.kernel.gat_keep_bits` of a
      dropout output (E, H, 1)) with ``keep_scale`` (the dropout's 1 / (1 - p)): the
      caller's mask -- GATConv passes its own ``nn.Dropout``'s draws, the reference's;
    * ``attn_drop`` > 0: a hashed mask keyed by ``seed`` (default: drawn from torch's
      default generator, so ``torch.manual_seed`` reproduces it) -- no (E, H) buffer, not
      torch's draws;
    * ``draw`` (:func:`dgl.kernel.dropout_draw`, taken for the (E, H) attention tensor):
      torch's own draws recomputed inside the kernels -- GATConv's default when
      :func:`dgl.kernel.dropout_draw_ok`."""
    gidx = graph if hasattr(graph, "in_csr") else graph._graph.get_immutable_gidx(feat_src.device)
    attn_drop = float(attn_drop)
    if draw is not None:
        return FusedGat.apply(gidx, feat_src, el, er, float(slope), 0.0, 0, None, None, draw)
    if keep is not None:
        if keep_scale is None:
            raise DGLError("fused_gat: keep needs keep_scale")
        return FusedGat.apply(gidx, feat_src, el, er, float(slope), 0.0, 0, keep,
                              float(keep_scale))
    if attn_drop > 0.0 and seed is None:
        seed = int(th.randint(0, 2 ** 62, (1,)).item())
    return FusedGat.apply(gidx, feat_src, el, er, float(slope), attn_drop, int(seed or 0))


class _AttnLogits(th.autograd.Function):
    """GATConv's el = (ft_src * attn_l).sum(-1), er = (ft_dst * attn_r).sum(-1)
    (gatconv.py:137-138) as one pass over the features each way (DGLMIGatAttnLogits /
    Backward) instead of a multiply and a reduction per side and, backward, a multiply,
    a multiply-reduce and an add per side.  ``feat_dst`` None: one table for both."""

    @staticmethod
    def forward(ctx, feat_src, attn_l, attn_r, feat_dst):
        el, er = K.attn_logits(feat_src, feat_dst, attn_l, attn_r)
        ctx.one = feat_dst is None
        ctx.save_for_backward(feat_src, attn_l, attn_r, feat_dst)
        return el, er

    @staticmethod
    def backward(ctx, g_el, g_er):
        feat_src, attn_l, attn_r, feat_dst = ctx.saved_tensors
        if g_el is None:
            g_el = feat_src.new_zeros(feat_src.shape[:2] + (1,))
        if g_er is None:
            n = feat_src.shape[0] if ctx.one else feat_dst.shape[0]
            g_er = feat_src.new_zeros((n, feat_src.shape[1], 1))
        gs, gd, gl, gr = K.attn_logits_backward(feat_src, None if ctx.one else feat_dst, attn_l,
                                                attn_r, g_el, g_er)
        return gs, gl, gr, gd


def attn_logits(feat_src, feat_dst, attn_l, attn_r):
    """(el, er), each (N, H, 1): GATConv's attention logits on the device
    (:class:`_AttnLogits`); ``feat_dst is feat_src``: one pass over one table."""
    one = feat_dst is feat_src
    return _AttnLogits.apply(feat_src, attn_l, attn_r, None if one else feat_dst)


class GatComposition(th.autograd.Function):
    """GATConv's unfused composition (gatconv.py:151-157: u_add_v, leaky_relu, edge_softmax,
    u_mul_e_sum) on the in-CSR position view, forward step by step -- the node-logit edge
    softmax, then u_mul_e_sum: the kernels and bits of the separate autograd Functions --
    and ONE fused backward: the fused GAT backward kernels (DGLMIFusedGatBackward: the
    destination- and source-side walks, or the edge-position path), fed the softmax's row
    statistics (DGLMIEdgeSoftmaxNodeLogitsForwardEx) and the output.  The step-by-step
    backward walks the edges five times (attention-gradient SDDMM, softmax backward, the
    two u_add_v gradient reductions, the u_mul_e_sum node gradient) and moves the E x H
    attention gradient and logit gradient through HBM; here the softmax identity
    sum_e a_e (ft_u . g_v) = g_v . rst_v gives each row's correction densely, the
    attention is recomputed where it is used, and no per-edge tensor is kept from the
    forward (the attention, E x H, is freed after u_mul_e_sum).  Equal to the step-by-step
    gradients within fp32 rounding (tests/test_nn_gpu.py).  ``draw``
    (dgl.kernel.dropout_draw over the (E, H) attention): GATConv's attention dropout with
    the module's own draws -- the attention times nn.Dropout's output on ones, written in
    walk order from the draws (DGLMIDropoutDrawScale), and the same draws recomputed by the
    backward walks (DGLMIFusedGatDrawBackward without slope aggregates)."""

    @staticmethod
    def forward(ctx, gidx, view, feat_src, el, er, slope, draw=None):
        ft, el, er = feat_src.contiguous(), el.contiguous(), er.contiguous()
        n_dst = view.num_dst
        H = el.shape[1]
        a = el.new_empty((view.number_of_edges(),) + tuple(el.shape[1:]))
        rmax = el.new_zeros((n_dst, H))
        rsum = el.new_ones((n_dst, H))
        K.edge_softmax_node_logits_forward_ex(view, el, er, slope, a, rmax, rsum)
        if draw is not None:  # dropout(a): a * (keep * scale), torch's order of operations
            K.dropout_draw_apply(draw, H, gidx.in_csr.data, a)
        rst = ft.new_empty((n_dst,) + tuple(ft.shape[1:]))
        K.binary_op_reduce("sum", "mul", view, SRC, EDGE, ft, a, rst)
        del a
        ctx.gidx, ctx.slope, ctx.draw = gidx, slope, draw
        ctx.save_for_backward(ft, el, er, rst, rmax, rsum)
        return rst

    @staticmethod
    def backward(ctx, grad):
        ft, el, er, rst, rmax, rsum = ctx.saved_tensors
        g_ft, g_el, g_er = th.empty_like(ft), th.empty_like(el), th.empty_like(er)
        K.fused_gat_backward(ctx.gidx, ft, el, er, ctx.slope, rst, rmax, rsum, grad.contiguous(),
                             g_ft, g_el, g_er, draw=ctx.draw)
        return None, None, g_ft, g_el, g_er, None, None


def gat_composition_ok(gidx, feat_src, el, er):
    """Whether GatComposition applies: 32-bit device CSRs with both directions, fp32 ft
    (N, H, D) whose head size the fused GAT kernels take, el / er (N, H, 1) with an H the
    fused edge softmax takes."""
    if not (feat_src.is_cuda and feat_src.dtype == th.float32 and feat_src.dim() == 3):
        return False
    n, h, d = feat_src.shape
    return (gidx.in_csr.bits == 32 and getattr(gidx, "out_csr", None) is not None
            and el.shape == (n, h, 1) and er.dim() == 3 and er.shape[1:] == (h, 1)
            and el.dtype == er.dtype == th.float32
            and K.fused_gat_supported(h, d) and K.edge_softmax_supported(h))


def gat_composition(gidx, view, feat_src, el, er, slope, draw=None):
    """rst = u_mul_e_sum(ft, edge_softmax(leaky_relu(u_add_v(el, er)))) with the fused
    backward (:class:`GatComposition`); ``view`` = gidx.position_view("in"); ``draw``:
    attention dropout with torch's own draws (dropout(edge_softmax(...)))."""
    return GatComposition.apply(gidx, view, feat_src, el, er, float(slope), draw)


# --------------------------------------------------------------------------- #
# R-GCN (hack: RgcnFirstLayer / RgcnSecondLayer, tensor.py:440-495;
# kernels binary_reduce_impl.cu:913-1246)
# --------------------------------------------------------------------------- #
class _TypedAggregate(th.autograd.Function):
    """out[v] = sum_e w_e * y[src_e] (+ bias + addend) on the relation-expanded
    graph with a CONSTANT per-edge weight w: the forward walks the in-CSR with w
    in in-CSR position order, the gradient of y walks the out-CSR with w in
    out-CSR position order (both streamed, both cached), and RelGraphConv's bias
    and self-loop term ride in the kernel epilogue instead of two extra passes
    over the output."""

    @staticmethod
    def forward(ctx, gidx, y, w, bias, addend, n):
        vin, w_in = gidx.position_operand(w, "in")
        out = y.new_empty((n, y.shape[1]))
        epi = None if bias is None and addend is None else (None, None, bias, addend)
        K.binary_op_reduce("sum", "mul", vin, SRC, EDGE, y, w_in, out, epilogue=epi)
        ctx.gidx, ctx.w = gidx, w
        ctx.has_bias, ctx.has_addend = bias is not None, addend is not None
        ctx.save_for_backward(y, out)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        y, out = ctx.saved_tensors
        g = grad_out.contiguous()
        gy = gb = ga = None
        if ctx.needs_input_grad[1]:
            vout, w_out = ctx.gidx.position_operand(ctx.w, "out")
            gy = th.empty_like(y)
            K.backward_lhs_binary_op_reduce("sum", "mul", vout, SRC, EDGE, y, w_out, out, g, gy)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            gb = g.sum(0)
        if ctx.has_addend and ctx.needs_input_grad[4]:
            ga = g
        return None, gy, None, gb, ga, None


def _typed_aggregate(graph, num_rels, y, norm, etypes, node_major=False, bias=None,
                     addend=None):
    """out[v] = sum_{e=(u->v)} norm_e * y[type_e * N + u] (or y[u * R + type_e] with
    ``node_major``): every relation in ONE load-balanced gather over the
    relation-expanded graph (no per-relation SpMMs, no per-edge weight products)."""
    gidx = graph._graph.typed_gidx(y.device, num_rels, etypes, node_major)
    n = graph.number_of_nodes()
    if norm is not None:
        w = norm.reshape(norm.shape[0], 1)
        if not w.requires_grad and w.is_cuda and gidx.eid_perm and y.dim() == 2:
            # constant norm: streamed in walk order, bias / addend in the epilogue
            return _TypedAggregate.apply(gidx, y, w, bias, addend, n)
        out = binary_reduce("sum", "mul", gidx, SRC, EDGE, y, w, n)
    else:
        out = copy_reduce("sum", gidx, SRC, y, n)
    if bias is not None:
        out = out + bias
    if addend is not None:
        out = out + addend
    return out


class _FusedRgcnLayer1(th.autograd.Function):
    """RelGraphConv's layer on the hack's layer-1 C entries with the prepared state
    (``DGLMIRgcnLayer1Ex`` / ``DGLMIRgcnLayer1BackwardEx``, fused aggregate-then-transform
    kernels): no (N, R * F_out) table Y = X [W_0 | ... | W_{R-1}] is
    written or gathered, and the self-loop message is one more MFMA pass over each
    tile's own rows, the bias added in the same output pass.  Gradients for x, the
    relation weights, the self-loop weight and the bias; the norm is constant."""

    @staticmethod
    def forward(ctx, gidx, et32, norm, x, w, loop_w, bias):
        ret = x.new_empty((gidx.num_dst, w.shape[2]))
        K.rgcn_layer1_ex(gidx, x, w, norm, ret, loop_weight=loop_w, bias=bias, etypes=et32)
        ctx.gidx, ctx.et32, ctx.norm = gidx, et32, norm
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, w, loop_w)
        return ret

    @staticmethod
    def backward(ctx, grad_out):
        x, w, loop_w = ctx.saved_tensors
        g = grad_out.contiguous()
        gx = gw = gl = gb = None
        if any(ctx.needs_input_grad[3:6]):
            # no input gradient wanted (a first layer over data): the walk skips its
            # MFMA passes and stores only the weight gradients' operand
            gx = th.empty_like(x) if ctx.needs_input_grad[3] else None
            gw = th.empty_like(w)
            gl = th.empty_like(loop_w) if loop_w is not None and ctx.needs_input_grad[5] else None
            K.rgcn_layer1_backward_ex(ctx.gidx, x, w, ctx.norm, loop_w, g, gx, gw, gl,
                                      etypes=ctx.et32)
        if ctx.has_bias and ctx.needs_input_grad[6]:
            gb = g.sum(0)
        return None, None, None, gx, gw, gl, gb


def rgcn_fused_route(graph, x, weight_shape, norm, etypes, self_loop=False):
    """(gidx, etypes int32, norm flat) when a RelGraphConv layer can run on the
    fused layer-1 C entries both ways (64-float rows gathered forward and backward,
    the relation and self-loop weights in LDS; DGLMIRgcnLayer1Ex / BackwardEx with a
    prepared state), else None.  The state (``kernel.rgcn_prepare``, ~6 values per
    edge) is built once per graph, device and etypes, and rebuilt when etypes is
    written in place; a different or rewritten norm only re-gathers its cached copies."""
    R, fi, fo = weight_shape
    mats = R + int(bool(self_loop))
    if not (x.is_cuda and x.dtype == th.float32 and x.dim() == 2 and x.shape[1] == fi
            and K.rgcn_fused_ok(fi, fo, mats) and K.rgcn_fused_ok(fo, fi, mats)):
        return None
    if norm is None or norm.requires_grad or not norm.is_cuda or norm.dtype != th.float32:
        return None
    if etypes is None or not isinstance(etypes, th.Tensor) or etypes.device != x.device:
        return None
    gi = graph._graph
    if x.shape[0] != graph.number_of_nodes() or gi.device_bits() != 32:
        return None
    if norm.numel() != graph.number_of_edges() or etypes.numel() != graph.number_of_edges():
        return None
    # the state depends on the relation ids only; a new or rewritten norm re-gathers
    # its cached copies (kernel.RgcnState.sync_norm) instead of rebuilding
    key = (str(x.device), int(R), etypes.data_ptr(), etypes._version, int(etypes.numel()))
    hit = gi.__dict__.get("_rgcn_fused")
    if hit is None or hit[0] != key:
        gidx = gi.get_immutable_gidx(x.device)
        et = etypes.reshape(-1)
        if et.numel() and (int(et.min()) < 0 or int(et.max()) >= R):
            raise DGLError("edge type out of range [0, %d)" % R)
        et32 = et.to(th.int32).contiguous()
        gi.__dict__.pop("_rgcn_fused", None)
        # rgcn_prepare releases the graph's previous state before allocating (~2 GB on C5)
        K.rgcn_prepare(gidx, norm.reshape(-1).contiguous(), R, layers=6, etypes=et32)
        # the cache holds the caller's etypes, so its address stays theirs
        hit = (key, gidx, et32, etypes)
        gi.__dict__["_rgcn_fused"] = hit
    return hit[1], hit[2], _flat_norm(gi, norm)


def _flat_norm(gi, norm):
    """``norm`` as one contiguous float per edge.  A contiguous norm is viewed (same
    storage: the prepared state's pointer / version check sees the caller's tensor); a
    non-contiguous one is copied ONCE per (tensor, version) and the copy reused, so
    RgcnState.sync_norm does not re-gather the state's norm copies on every call.  The
    cache holds the source's storage owner only by a weak reference whose callback
    drops the entry -- and the E-float copy -- the moment the source is freed."""
    flat = norm.reshape(-1)
    if flat.is_contiguous():
        return flat
    key = (norm.data_ptr(), norm._version, tuple(norm.shape), tuple(norm.stride()))
    owner = norm._base if norm._base is not None else norm
    hit = gi.__dict__.get("_rgcn_norm_flat")
    if hit is not None and hit[0] == key and hit[1]() is owner:
        return hit[2]
    copy = flat.contiguous()
    d = gi.__dict__

    def drop(ref):
        ent = d.get("_rgcn_norm_flat")
        if ent is not None and ent[1] is ref:
            del d["_rgcn_norm_flat"]
    d["_rgcn_norm_flat"] = (key, weakref.ref(owner, drop), copy)
    return copy


def rgcn_fused_layer1(route, x, weight, loop_weight=None, bias=None):
    gidx, et32, nf = route
    return _FusedRgcnLayer1.apply(gidx, et32, nf, x.contiguous(), weight.contiguous(),
                                  None if loop_weight is None else loop_weight.contiguous(), bias)


def rgcn_layer0(graph, weight, norm, etypes=None):
    """Layer with one-hot (node id) input: ret[v] = sum_e W[type_e, u] * norm_e.

    weight (R, N, F_out).  The hack's backward overwrites instead of accumulating
    when a (src, type) pair repeats (binary_reduce_impl.cu:1004); here the
    gradient is the exact one (autograd through the gather)."""
    R, n, f = weight.shape
    return _typed_aggregate(graph, R, weight.reshape(R * n, f), norm, etypes)


def rgcn_layer1(graph, x, weight, norm, etypes=None):
    """ret[v] = sum_e (x[u] @ W[type_e]) * norm_e.

    The per-edge (F_in x F_out) products of the hack's kernel (binary_reduce_impl.cu:
    1050-1117) become ONE dense GEMM Y = X [W_0 | ... | W_{R-1}] (N x R*F_out, MFMA
    via hipBLASLt) plus one typed gather over rows u * R + type; the hack also drops
    the weight gradient (tensor.py:493), autograd keeps it."""
    R, fi, fo = weight.shape
    y = project(x, weight.permute(1, 0, 2).reshape(fi, R * fo))  # (N, R * F_out)
    return _typed_aggregate(graph, R, y.view(x.shape[0] * R, fo), norm, etypes, node_major=True)
