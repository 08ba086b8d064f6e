"""GatedGraphConv (``python/dgl/nn/pytorch/conv/gatedgraphconv.py:10-98``).

Per step: a_v = sum_{e=(u->v)} Linear_{type_e}(h_u), then h <- GRUCell(a, h).
The reference runs one masked ``apply_edges`` per edge type (an E x out
message tensor, each edge's Linear on its own row) and a copy_e sum.  Here
all types are ONE GEMM over the nodes, h [W_0^T | ... | W_{R-1}^T] + [b_0 | ...]
(N x R*out on MFMA), and ONE typed gather kernel over the relation-expanded
graph (rows u * R + type_e; the R-GCN aggregation, ``dgl.backend._typed_aggregate``)
-- per edge the bytes of one output row, no per-edge message tensor.
``fused = False`` restores the reference's per-type apply_edges.
"""
import torch as th
from torch import nn
from torch.nn import init

from .... import backend as B
from .... import function as fn


class GatedGraphConv(nn.Module):
    def __init__(self, in_feats, out_feats, n_steps, n_etypes, bias=True):
        super(GatedGraphConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._n_steps = n_steps
        self._n_etypes = n_etypes
        self.linears = nn.ModuleList([nn.Linear(out_feats, out_feats) for _ in range(n_etypes)])
        self.gru = nn.GRUCell(out_feats, out_feats, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        gain = init.calculate_gain("relu")
        self.gru.reset_parameters()
        for linear in self.linears:
            init.xavier_normal_(linear.weight, gain=gain)
            init.zeros_(linear.bias)

    def forward(self, graph, feat, etypes):
        graph = graph.local_var()
        zero_pad = feat.new_zeros((feat.shape[0], self._out_feats - feat.shape[1]))
        feat = th.cat([feat, zero_pad], -1)
        fused = getattr(self, "fused", True) and feat.is_cuda and feat.dtype == th.float32
        n, R, fo = feat.shape[0], self._n_etypes, self._out_feats
        if fused:
            w = th.cat([lin.weight.t() for lin in self.linears], 1)  # (out, R * out)
            b = th.cat([lin.bias for lin in self.linears])
        for _ in range(self._n_steps):
            if fused:
                y = B.project(feat, w, b)  # (N, R * out): row u * R + t = Linear_t(h_u)
                a = B._typed_aggregate(graph, R, y.view(n * R, fo), None, etypes,
                                       node_major=True)
            else:
                graph.ndata["h"] = feat
                for i in range(R):
                    eids = (etypes == i).nonzero().view(-1)
                    if len(eids) > 0:
                        graph.apply_edges(
                            lambda edges, i=i: {"W_e*h": self.linears[i](edges.src["h"])},
                            eids)
                graph.update_all(fn.copy_e("W_e*h", "m"), fn.sum("m", "a"))
                a = graph.ndata.pop("a")
            feat = self.gru(a, feat)
        return feat
