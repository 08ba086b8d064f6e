"""AGNNConv (``python/dgl/nn/pytorch/conv/agnnconv.py:10-74``).

p_uv = edge_softmax(beta * cos(h_u, h_v)), h'_v = sum_u p_uv h_u: the
``u_dot_v`` SDDMM kernel on L2-normalised rows, the fused edge-softmax
kernels and ``u_mul_e_sum`` (attention broadcast over the feature dim) --
all builtins on the HIP path.
"""
import torch as th
from torch import nn
from torch.nn import functional as F

from .... import function as fn
from ..softmax import edge_softmax
from .gatconv import expand_as_pair


class AGNNConv(nn.Module):
    def __init__(self, init_beta=1., learn_beta=True):
        super(AGNNConv, self).__init__()
        if learn_beta:
            self.beta = nn.Parameter(th.Tensor([init_beta]))
        else:
            self.register_buffer("beta", th.Tensor([init_beta]))

    def forward(self, graph, feat):
        graph = graph.local_var()
        feat_src, feat_dst = expand_as_pair(feat)
        graph.srcdata["h"] = feat_src
        graph.srcdata["norm_h"] = F.normalize(feat_src, p=2, dim=-1)
        if isinstance(feat, tuple):
            graph.dstdata["norm_h"] = F.normalize(feat_dst, p=2, dim=-1)
        graph.apply_edges(fn.u_dot_v("norm_h", "norm_h", "cos"))
        cos = graph.edata.pop("cos")
        graph.edata["p"] = edge_softmax(graph, self.beta * cos)
        graph.update_all(fn.u_mul_e("h", "p", "m"), fn.sum("m", "h"))
        return graph.dstdata.pop("h")
