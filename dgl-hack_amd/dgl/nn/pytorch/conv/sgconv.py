"""SGConv (``python/dgl/nn/pytorch/conv/sgconv.py:10-103``).

(D^-1/2 A D^-1/2)^k X, then one Linear.  Each hop is ONE copy_u_sum launch
with the destination-side D^-1/2 in the kernel's epilogue
(``dgl.backend.gcn_aggregate``); the source-side scaling is a row multiply
on the input.  ``cached`` keeps the propagated features as the reference
does.  Note the reference uses the IN-degree on both sides (sgconv.py:85-88).
"""
import torch as th
from torch import nn

from .... import backend as B
from .... import function as fn


def propagate_sym(graph, feat, norm, steps, fused=True):
    """``steps`` hops of feat <- norm * (A (norm * feat)) (norm: (N,) float32)."""
    if fused and feat.dim() == 2 and feat.dtype == th.float32 and feat.is_cuda:
        gidx = graph._graph.get_immutable_gidx(feat.device)
        n = graph.number_of_dst_nodes()
        for _ in range(steps):
            feat = B.gcn_aggregate(gidx, feat * norm.view(-1, 1), norm, None, n)
        return feat
    shp = norm.shape + (1,) * (feat.dim() - 1)
    norm = th.reshape(norm, shp)
    for _ in range(steps):
        feat = feat * norm
        graph.ndata["h"] = feat
        graph.update_all(fn.copy_u("h", "m"), fn.sum("m", "h"))
        feat = graph.ndata.pop("h")
        feat = feat * norm
    return feat


def in_degree_norm(graph, device):
    """in_degrees().clamp(min=1) ** -0.5 from the cached device CSR."""
    return th.pow(graph._device_degrees(device, "in").float().clamp(min=1), -0.5)


class SGConv(nn.Module):
    def __init__(self, in_feats, out_feats, k=1, cached=False, bias=True, norm=None):
        super(SGConv, self).__init__()
        self.fc = nn.Linear(in_feats, out_feats, bias=bias)
        self._cached = cached
        self._cached_h = None
        self._k = k
        self.norm = norm
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.fc.weight)
        if self.fc.bias is not None:
            nn.init.zeros_(self.fc.bias)

    def forward(self, graph, feat):
        graph = graph.local_var()
        if self._cached_h is not None:
            feat = self._cached_h
        else:
            norm = in_degree_norm(graph, feat.device)
            feat = propagate_sym(graph, feat, norm, self._k, getattr(self, "fused", True))
            if self.norm is not None:
                feat = self.norm(feat)
            if self._cached:
                self._cached_h = feat
        return self.fc(feat)
