"""Edge softmax (``python/dgl/nn/pytorch/softmax.py:15-193``).

Same decomposition as the reference: per destination the max of the incoming
logits is subtracted before ``exp`` (``copy_e`` max, ``e_sub_v``), the sum of
the exponentials divides them (``copy_e`` sum, ``e_div_v``), and the
backward is ``grad_s - out * sum_dst(out * grad_out)``
(``softmax.py:86-114``).

With 1, 2, 4, 8 or 16 values per edge the whole forward is one fused kernel
pair (``kernels_softmax.hip``: per destination an online running max / sum of
exponentials over its in-edges, then one per-edge normalisation pass in
edge-id order) and so is the backward; other shapes run the reference's
decomposition, each step one g-SpMM / g-SDDMM kernel call.  ``FUSED = False``
forces the decomposition.
"""
import torch as th

from ... import backend as F
from ... import kernel as K
from ...function import TargetCode
from ...graph import ALL, is_all, _PartialIndex

__all__ = ["edge_softmax"]


FUSED = True


class FusedEdgeSoftmax(th.autograd.Function):
    @staticmethod
    def forward(ctx, gidx, score):
        score = score.contiguous()
        out = th.empty_like(score)
        K.edge_softmax_forward(gidx, score, out)
        ctx.gidx = gidx
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        out, = ctx.saved_tensors
        grad = th.empty_like(out)
        K.edge_softmax_backward(ctx.gidx, out, grad_out.contiguous(), grad)
        return None, grad


class FusedLeakyEdgeSoftmax(th.autograd.Function):
    """edge_softmax(leaky_relu(x)) with the activation inside the softmax's passes: the
    activated logits are never written, and the backward multiplies by leaky_relu'(x)
    where it writes the gradient (torch's operations: bit-identical to the two steps)."""

    @staticmethod
    def forward(ctx, gidx, x, slope):
        x = x.contiguous()
        out = th.empty_like(x)
        K.edge_softmax_leaky_forward(gidx, x, slope, out)
        ctx.gidx, ctx.slope = gidx, slope
        ctx.save_for_backward(out, x)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        out, x = ctx.saved_tensors
        grad = th.empty_like(out)
        K.edge_softmax_leaky_backward(ctx.gidx, out, grad_out.contiguous(), x, ctx.slope, grad)
        return None, grad, None


class FusedNodeLogitEdgeSoftmax(th.autograd.Function):
    """edge_softmax(leaky_relu(u_add_v(el, er))) with the logits computed where the
    softmax reads them (never stored); the backward writes their gradient and hands it to
    u_add_v's own gradient kernels (BinaryReduce.backward's calls) -- the three-step
    composition's bits."""

    @staticmethod
    def forward(ctx, gidx, el, er, slope):
        el, er = el.contiguous(), er.contiguous()
        out = el.new_empty((gidx.number_of_edges(),) + tuple(el.shape[1:]))
        K.edge_softmax_node_logits_forward(gidx, el, er, slope, out)
        ctx.gidx, ctx.slope = gidx, slope
        ctx.save_for_backward(out, el, er)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        out, el, er = ctx.saved_tensors
        gidx = ctx.gidx
        gs = th.empty_like(out)
        K.edge_softmax_node_logits_backward(gidx, out, grad_out.contiguous(), el, er, ctx.slope, gs)
        g_el = g_er = None
        if ctx.needs_input_grad[1]:
            g_el = th.empty_like(el)
            K.backward_lhs_binary_op_reduce("none", "add", gidx, TargetCode.SRC, TargetCode.DST,
                                            el, er, gs, gs, g_el)
        if ctx.needs_input_grad[2]:
            g_er = th.empty_like(er)
            K.backward_rhs_binary_op_reduce("none", "add", gidx, TargetCode.SRC, TargetCode.DST,
                                            el, er, gs, gs, g_er)
        return None, g_el, g_er, None


def _apply_node_logits(gidx, el, er, n_nodes, slope):
    """edge_softmax(leaky_relu(u_add_v(el, er))) -- one fused pair without stored
    logits where the softmax is fused and el / er have the same per-node shape, else the
    three steps."""
    m = gidx.number_of_edges()
    if (el.shape[1:] == er.shape[1:] and er.dtype == el.dtype and er.is_cuda and
            _fusable_as(gidx, (m,) + tuple(el.shape[1:]), el.dtype, el.is_cuda)):
        return FusedNodeLogitEdgeSoftmax.apply(gidx, el, er, float(slope))
    e = F.binary_reduce("none", "add", gidx, TargetCode.SRC, TargetCode.DST, el, er, m)
    return _apply_leaky(gidx, e, n_nodes, slope)


def _fusable_as(gidx, shape, dtype, is_cuda):
    h = 1
    for d in shape[1:]:
        h *= d
    return (FUSED and dtype == th.float32 and K.edge_softmax_supported(h) and
            shape[0] == gidx.number_of_edges() and is_cuda)


def _fusable(gidx, logits):
    return _fusable_as(gidx, logits.shape, logits.dtype, logits.is_cuda)


def _apply_leaky(gidx, x, n_nodes, slope):
    """edge_softmax(leaky_relu(x, slope)) -- one fused pair where the softmax is fused,
    else the two steps."""
    if _fusable(gidx, x):
        return FusedLeakyEdgeSoftmax.apply(gidx, x, float(slope))
    return _apply(gidx, th.nn.functional.leaky_relu(x, slope), n_nodes)


def _apply(gidx, logits, n_nodes):
    if _fusable(gidx, logits):
        return FusedEdgeSoftmax.apply(gidx, logits)
    return EdgeSoftmax.apply(gidx, logits, n_nodes)


class EdgeSoftmax(th.autograd.Function):
    @staticmethod
    def forward(ctx, gidx, score, n_nodes):
        n_edges = score.shape[0]
        score = score.contiguous()
        smax = F.copy_reduce("max", gidx, TargetCode.EDGE, score, n_nodes)
        out = F.binary_reduce("none", "sub", gidx, TargetCode.EDGE, TargetCode.DST, score, smax,
                              n_edges)
        out = th.exp(out)
        out_sum = F.copy_reduce("sum", gidx, TargetCode.EDGE, out, n_nodes)
        out = F.binary_reduce("none", "div", gidx, TargetCode.EDGE, TargetCode.DST, out, out_sum,
                              n_edges)
        ctx.backward_cache = (n_nodes, n_edges, gidx)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        n_nodes, n_edges, gidx = ctx.backward_cache
        out, = ctx.saved_tensors
        grad_s = (out * grad_out).contiguous()
        accum = F.copy_reduce("sum", gidx, TargetCode.EDGE, grad_s, n_nodes)
        out = F.binary_reduce("none", "mul", gidx, TargetCode.EDGE, TargetCode.DST, out, accum,
                              n_edges)
        return None, grad_s - out, None


def edge_softmax(graph, logits, eids=ALL):
    """Softmax over the incoming edges of every node.

    ``logits`` has shape (E, *, 1) (or (E,)); with ``eids`` given, only those
    edges take part and the result has their rows (``softmax.py:117-193``).
    """
    if is_all(eids):
        gidx = graph._graph.get_immutable_gidx(logits.device)
        return _apply(gidx, logits, graph.number_of_nodes())
    import numpy as np
    eids_np = eids.detach().cpu().numpy().astype(np.int64) if isinstance(eids, th.Tensor) \
        else np.asarray(eids, np.int64)
    src, dst, _ = graph._graph.edges()
    # local edge ids 0..k-1 in the order of `eids`, like edge_subgraph
    sub = _PartialIndex(graph.number_of_nodes(), src[eids_np], dst[eids_np],
                        np.arange(len(eids_np), dtype=np.int64))
    gidx = sub.get_immutable_gidx(logits.device)
    return _apply(gidx, logits, graph.number_of_nodes())
