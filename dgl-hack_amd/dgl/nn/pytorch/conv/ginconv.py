"""GINConv (``python/dgl/nn/pytorch/conv/ginconv.py:10-82``).

rst = (1 + eps) * h_dst + aggregate(h_src), then ``apply_func``.  For the
'sum' and 'mean' aggregators on 2-D float32 features the (1 + eps) * h_dst
term (and the mean's division by the degree) runs in the copy_u_sum
kernel's epilogue (``dgl.backend.gcn_aggregate``), so the layer is one
load-balanced launch; 'max' is copy_u_max (tie-mask gradient) plus the
residual.  ``fused = False`` restores the reference's update_all order.
"""
import torch as th
from torch import nn

from .... import backend as B
from .... import function as fn
from .gatconv import expand_as_pair


class GINConv(nn.Module):
    def __init__(self, apply_func, aggregator_type, init_eps=0, learn_eps=False):
        super(GINConv, self).__init__()
        self.apply_func = apply_func
        reducers = {"sum": fn.sum, "max": fn.max, "mean": fn.mean}
        if aggregator_type not in reducers:
            raise KeyError("Aggregator type {} not recognized.".format(aggregator_type))
        self._aggregator_type = aggregator_type
        self._reducer = reducers[aggregator_type]
        if learn_eps:
            self.eps = nn.Parameter(th.FloatTensor([init_eps]))
        else:
            self.register_buffer("eps", th.FloatTensor([init_eps]))

    def forward(self, graph, feat):
        graph = graph.local_var()
        feat_src, feat_dst = expand_as_pair(feat)
        n_dst = graph.number_of_dst_nodes()
        if (getattr(self, "fused", True) and self._aggregator_type in ("sum", "mean")
                and feat_src.dim() == 2 and feat_src.dtype == th.float32 and feat_src.is_cuda):
            gidx = graph._graph.get_immutable_gidx(feat_src.device)
            div = None
            if self._aggregator_type == "mean":
                div = graph._device_degrees(feat_src.device, "in").float().clamp(min=1)
            rst = B.gcn_aggregate(gidx, feat_src, None, None, n_dst, row_div=div,
                                  addend=(1 + self.eps) * feat_dst[:n_dst])
        else:
            graph.srcdata["h"] = feat_src
            graph.update_all(fn.copy_u("h", "m"), self._reducer("m", "neigh"))
            rst = (1 + self.eps) * feat_dst + graph.dstdata["neigh"]
        if self.apply_func is not None:
            rst = self.apply_func(rst)
        return rst
