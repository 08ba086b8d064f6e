"""TAGConv (``python/dgl/nn/pytorch/conv/tagconv.py:9-101``).

[X, AX, A^2X, ..., A^kX] (A = D^-1/2 A D^-1/2, in-degree norm on both sides)
concatenated, then one Linear.  Each hop is one copy_u_sum launch with the
destination-side norm in its epilogue (``sgconv.propagate_sym``).
"""
import torch as th
from torch import nn

from .sgconv import in_degree_norm, propagate_sym


class TAGConv(nn.Module):
    def __init__(self, in_feats, out_feats, k=2, bias=True, activation=None):
        super(TAGConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._k = k
        self._activation = activation
        self.lin = nn.Linear(in_feats * (self._k + 1), out_feats, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_normal_(self.lin.weight, gain=gain)

    def forward(self, graph, feat):
        graph = graph.local_var()
        norm = in_degree_norm(graph, feat.device)
        fused = getattr(self, "fused", True)
        fstack = [feat]
        for _ in range(self._k):
            fstack.append(propagate_sym(graph, fstack[-1], norm, 1, fused))
        rst = self.lin(th.cat(fstack, dim=-1))
        if self._activation is not None:
            rst = self._activation(rst)
        return rst
