"""NNConv (``python/dgl/nn/pytorch/conv/nnconv.py:11-121``).

Edge-conditioned convolution: per edge a (d_in x d_out) matrix from
``edge_func``; messages h_u[:, None] * W_e reduced by ``u_mul_e`` with
broadcasting (h: (N, d_in, 1) x w: (E, d_in, d_out) -> (N, d_in, d_out)),
then summed over d_in -- the reference's order, on the broadcast
load-balanced kernel (per edge d_in x d_out products, no message tensor).
"""
import torch as th
from torch import nn

from .... import function as fn
from .gatconv import Identity, expand_as_pair


class NNConv(nn.Module):
    def __init__(self, in_feats, out_feats, edge_func, aggregator_type, residual=False,
                 bias=True):
        super(NNConv, self).__init__()
        self._in_src_feats, self._in_dst_feats = expand_as_pair(in_feats)
        self._out_feats = out_feats
        self.edge_nn = edge_func
        reducers = {"sum": fn.sum, "mean": fn.mean, "max": fn.max}
        if aggregator_type not in reducers:
            raise KeyError("Aggregator type {} not recognized: ".format(aggregator_type))
        self.reducer = reducers[aggregator_type]
        self._aggre_type = aggregator_type
        if residual:
            if self._in_dst_feats != out_feats:
                self.res_fc = nn.Linear(self._in_dst_feats, out_feats, bias=False)
            else:
                self.res_fc = Identity()
        else:
            self.register_buffer("res_fc", None)
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_buffer("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        if self.bias is not None:
            nn.init.zeros_(self.bias)
        if isinstance(self.res_fc, nn.Linear):
            nn.init.xavier_normal_(self.res_fc.weight, gain=gain)

    def forward(self, graph, feat, efeat):
        graph = graph.local_var()
        feat_src, feat_dst = expand_as_pair(feat)
        graph.srcdata["h"] = feat_src.unsqueeze(-1)  # (N, d_in, 1)
        graph.edata["w"] = self.edge_nn(efeat).view(-1, self._in_src_feats, self._out_feats)
        graph.update_all(fn.u_mul_e("h", "w", "m"), self.reducer("m", "neigh"))
        rst = graph.dstdata["neigh"].sum(dim=1)  # (N, d_out)
        if self.res_fc is not None:
            rst = rst + self.res_fc(feat_dst)
        if self.bias is not None:
            rst = rst + self.bias
        return rst
