"""APPNPConv (``python/dgl/nn/pytorch/conv/appnpconv.py:9-73``).

k hops of  h <- (1 - alpha) * D^-1/2 A D^-1/2 h + alpha * h0.  Without an
active edge dropout the reference's per-edge weight is all ones, so each hop
is ONE copy_u_sum launch whose epilogue applies (1 - alpha) * D^-1/2 and adds
alpha * h0 (``dgl.backend.gcn_aggregate``) -- no E-sized ones tensor, no
u_mul_e, no two passes over the output.  With edge dropout active in
training the reference's u_mul_e_sum over the dropped weights runs.
"""
import torch as th
from torch import nn

from .... import backend as B
from .... import function as fn
from .sgconv import in_degree_norm


class APPNPConv(nn.Module):
    def __init__(self, k, alpha, edge_drop=0.):
        super(APPNPConv, self).__init__()
        self._k = k
        self._alpha = alpha
        self.edge_drop = nn.Dropout(edge_drop)

    def forward(self, graph, feat):
        graph = graph.local_var()
        norm = in_degree_norm(graph, feat.device)
        feat_0 = feat
        dropping = self.training and self.edge_drop.p > 0
        if (not dropping and getattr(self, "fused", True) and feat.dim() == 2
                and feat.dtype == th.float32 and feat.is_cuda):
            gidx = graph._graph.get_immutable_gidx(feat.device)
            n = graph.number_of_nodes()
            scale = (1 - self._alpha) * norm
            tail = self._alpha * feat_0
            for _ in range(self._k):
                feat = B.gcn_aggregate(gidx, feat * norm.view(-1, 1), scale, None, n,
                                       addend=tail)
            return feat
        norm = th.reshape(norm, norm.shape + (1,) * (feat.dim() - 1))
        for _ in range(self._k):
            feat = feat * norm
            graph.ndata["h"] = feat
            graph.edata["w"] = self.edge_drop(
                th.ones(graph.number_of_edges(), 1, device=feat.device))
            graph.update_all(fn.u_mul_e("h", "w", "m"), fn.sum("m", "h"))
            feat = graph.ndata.pop("h")
            feat = feat * norm
            feat = (1 - self._alpha) * feat + self._alpha * feat_0
        return feat
