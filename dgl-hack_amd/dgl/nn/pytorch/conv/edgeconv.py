"""EdgeConv (``python/dgl/nn/pytorch/conv/edgeconv.py:9-98``).

The reference materialises one message per edge,
e_uv = theta(x_v - x_u) + phi(x_u)  (E x out floats through two Linears on
E rows), then max-reduces.  Both maps are affine, so
e_uv = [x_v W_t^T + b_t + b_p] + [x_u (W_p - W_t)^T]  =  a_v + b_u, and
max_u e_uv = a_v + max_u b_u:  two node-level GEMMs (MFMA) and ONE
copy_u_max kernel, no per-edge tensor.  A destination with no in-edge keeps
the max reducer's identity (-FLT_MAX), as the reference.

Gradient, as the reference's max backward: every edge whose message ties the
maximum gets grad_out (``cpu/functor.h`` / ``binary_reduce_common.h`` BackwardCall
for max).  So b gets the copy_u_max tie-mask gradient, and a_v gets grad_out_v
times the number of tied in-edges of v: 1 when the maximum is unique, 0 with no
in-edge, more on exact ties (duplicate edges, repeated feature values).  The
tie counts come from one extra tie-mask pass over ones; only when that shows a
destination with several ties is the per-edge comparison materialised.

``batch_norm=True`` (a BatchNorm over the per-edge messages) needs the
messages, and ``fused = False`` restores the reference order -- both run the
message UDF + copy_e max.
"""
import torch as th
from torch import nn

from .... import function as fn
from .... import kernel as K
from ....backend import SRC
from .gatconv import expand_as_pair


class _PlusNeighbourMax(th.autograd.Function):
    """out[v] = a[v] + max_{u->v} b[u] (copy_u_max + a broadcast add)."""

    @staticmethod
    def forward(ctx, gidx, a, b):
        m = b.new_empty((gidx.in_csr.num_rows, b.shape[1]))
        K.copy_reduce("max", gidx, SRC, b, m)
        ctx.gidx = gidx
        ctx.save_for_backward(b, m)
        return a + m

    @staticmethod
    def backward(ctx, g):
        b, m = ctx.saved_tensors
        gidx = ctx.gidx
        g = g.contiguous()
        gb = th.empty_like(b)
        K.backward_copy_reduce("max", gidx, SRC, b, m, g, gb)
        # tie counts per (v, feature): sum over sources of the tie mask
        per_src = th.empty_like(b)
        K.backward_copy_reduce("max", gidx, SRC, b, m, th.ones_like(g), per_src)
        deg = gidx.in_csr.degrees()
        has_edge = (deg > 0).to(g.dtype).view(-1, 1)
        if bool((per_src.sum(0) == has_edge.sum()).all()):
            ties = has_edge
        else:
            dst = th.repeat_interleave(th.arange(deg.shape[0], device=g.device), deg.long())
            src = gidx.in_csr.indices.long()
            ties = th.zeros_like(m).index_add_(0, dst, (b[src] == m[dst]).to(m.dtype))
        return None, g * ties, gb


class EdgeConv(nn.Module):
    def __init__(self, in_feat, out_feat, batch_norm=False):
        super(EdgeConv, self).__init__()
        self.batch_norm = batch_norm
        self.theta = nn.Linear(in_feat, out_feat)
        self.phi = nn.Linear(in_feat, out_feat)
        if batch_norm:
            self.bn = nn.BatchNorm1d(out_feat)

    def message(self, edges):
        theta_x = self.theta(edges.dst["x"] - edges.src["x"])
        phi_x = self.phi(edges.src["x"])
        return {"e": theta_x + phi_x}

    def forward(self, g, h):
        g = g.local_var()
        h_src, h_dst = expand_as_pair(h)
        if not self.batch_norm and getattr(self, "fused", True) and h_src.is_cuda:
            w_t, w_p = self.theta.weight, self.phi.weight
            a = nn.functional.linear(h_dst, w_t, self.theta.bias + self.phi.bias)
            b = nn.functional.linear(h_src, w_p - w_t)
            gidx = g._graph.get_immutable_gidx(h_src.device)
            return _PlusNeighbourMax.apply(gidx, a[:g.number_of_dst_nodes()].contiguous(),
                                           b.contiguous())
        g.srcdata["x"] = h_src
        g.dstdata["x"] = h_dst
        if not self.batch_norm:
            g.update_all(self.message, fn.max("e", "x"))
        else:
            g.apply_edges(self.message)
            g.edata["e"] = self.bn(g.edata["e"])
            g.update_all(fn.copy_e("e", "e"), fn.max("e", "x"))
        return g.dstdata["x"]
