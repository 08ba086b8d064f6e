"""GMMConv (``python/dgl/nn/pytorch/conv/gmmconv.py:11-131``).

Gaussian kernel weights w_e,k = exp(-1/2 sum_d ((p_e,d - mu_k,d) inv_sigma_k,d)^2)
computed per edge in torch, then ONE broadcast ``u_mul_e`` reduce kernel
(h: (N, K, out) x w: (E, K, 1), the weight broadcast over the feature dim)
and a sum over the K kernels, plus the residual and bias.
"""
import torch as th
from torch import nn
from torch.nn import init

from .... import function as fn
from .gatconv import Identity, expand_as_pair


class GMMConv(nn.Module):
    def __init__(self, in_feats, out_feats, dim, n_kernels, aggregator_type="sum",
                 residual=False, bias=True):
        super(GMMConv, self).__init__()
        self._in_src_feats, self._in_dst_feats = expand_as_pair(in_feats)
        self._out_feats = out_feats
        self._dim = dim
        self._n_kernels = n_kernels
        reducers = {"sum": fn.sum, "mean": fn.mean, "max": fn.max}
        if aggregator_type not in reducers:
            raise KeyError("Aggregator type {} not recognized.".format(aggregator_type))
        self._reducer = reducers[aggregator_type]
        self.mu = nn.Parameter(th.Tensor(n_kernels, dim))
        self.inv_sigma = nn.Parameter(th.Tensor(n_kernels, dim))
        self.fc = nn.Linear(self._in_src_feats, n_kernels * out_feats, bias=False)
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
        gain = init.calculate_gain("relu")
        init.xavier_normal_(self.fc.weight, gain=gain)
        if isinstance(self.res_fc, nn.Linear):
            init.xavier_normal_(self.res_fc.weight, gain=gain)
        init.normal_(self.mu.data, 0, 0.1)
        init.constant_(self.inv_sigma.data, 1)
        if self.bias is not None:
            init.zeros_(self.bias.data)

    def forward(self, graph, feat, pseudo):
        graph = graph.local_var()
        feat_src, feat_dst = expand_as_pair(feat)
        graph.srcdata["h"] = self.fc(feat_src).view(-1, self._n_kernels, self._out_feats)
        E = graph.number_of_edges()
        gaussian = -0.5 * ((pseudo.view(E, 1, self._dim)
                            - self.mu.view(1, self._n_kernels, self._dim)) ** 2)
        gaussian = gaussian * (self.inv_sigma.view(1, self._n_kernels, self._dim) ** 2)
        graph.edata["w"] = th.exp(gaussian.sum(dim=-1, keepdim=True))  # (E, K, 1)
        graph.update_all(fn.u_mul_e("h", "w", "m"), self._reducer("m", "h"))
        rst = graph.dstdata["h"].sum(1)
        if self.res_fc is not None:
            rst = rst + self.res_fc(feat_dst)
        if self.bias is not None:
            rst = rst + self.bias
        return rst
