"""SAGEConv (``python/dgl/nn/pytorch/conv/sageconv.py:11-161``).

Same parameters, initialisation and aggregators ('mean', 'gcn', 'pool',
'lstm') as the reference.  The neighbour projection ``fc_neigh`` is linear, so
for 'mean' and 'gcn' it runs BEFORE the aggregation when that shrinks the
rows the kernel gathers (in_src_feats > out_feats), and the aggregation's
division by the degree, the 'gcn' self term and fc_neigh's bias ride in the
copy_u_sum kernel's epilogue (``dgl.backend.gcn_aggregate``): one load-balanced
launch per layer instead of copy_u_sum + a mean pass + a divide + a GEMM over
N x in_src_feats.  'pool' is a copy_u_max (the tie-mask gradient kernel);
'lstm' is the reference's UDF reducer on degree buckets.  ``fused = False``
on the module restores the reference's step order (update_all + nn.Linear).
"""
import torch as th
from torch import nn
from torch.nn import functional as F

from .... import backend as B
from .... import function as fn
from ...._ffi import DGLError
from .gatconv import expand_as_pair


class SAGEConv(nn.Module):
    def __init__(self, in_feats, out_feats, aggregator_type, feat_drop=0., bias=True,
                 norm=None, activation=None):
        super(SAGEConv, self).__init__()
        self._in_src_feats, self._in_dst_feats = expand_as_pair(in_feats)
        self._out_feats = out_feats
        self._aggre_type = aggregator_type
        self.norm = norm
        self.feat_drop = nn.Dropout(feat_drop)
        self.activation = activation
        if aggregator_type not in ("mean", "gcn", "pool", "lstm"):
            raise KeyError("Aggregator type {} not recognized.".format(aggregator_type))
        if aggregator_type == "pool":
            self.fc_pool = nn.Linear(self._in_src_feats, self._in_src_feats)
        if aggregator_type == "lstm":
            self.lstm = nn.LSTM(self._in_src_feats, self._in_src_feats, batch_first=True)
        if aggregator_type != "gcn":
            self.fc_self = nn.Linear(self._in_dst_feats, out_feats, bias=bias)
        self.fc_neigh = nn.Linear(self._in_src_feats, out_feats, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        if self._aggre_type == "pool":
            nn.init.xavier_uniform_(self.fc_pool.weight, gain=gain)
        if self._aggre_type == "lstm":
            self.lstm.reset_parameters()
        if self._aggre_type != "gcn":
            nn.init.xavier_uniform_(self.fc_self.weight, gain=gain)
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=gain)

    def _lstm_reducer(self, nodes):
        m = nodes.mailbox["m"]  # (bucket, degree, D)
        h0 = m.new_zeros((1, m.shape[0], self._in_src_feats))
        _, (rst, _) = self.lstm(m, (h0, h0))
        return {"neigh": rst.squeeze(0)}

    def _fusable(self, feat_src):
        return (getattr(self, "fused", True) and self._aggre_type in ("mean", "gcn")
                and feat_src.dim() == 2 and feat_src.dtype == th.float32 and feat_src.is_cuda)

    def _fused_neigh(self, graph, feat_src, feat_dst):
        """fc_neigh(aggregate(feat_src)) as one copy_u_sum launch with its epilogue."""
        gidx = graph._graph.get_immutable_gidx(feat_src.device)
        n_dst = graph.number_of_dst_nodes()
        degs = graph._device_degrees(feat_src.device, "in").float()
        w, b = self.fc_neigh.weight, self.fc_neigh.bias
        pre = self._in_src_feats > self._out_feats
        x = B.project(feat_src, w.t()) if pre else feat_src
        if self._aggre_type == "mean":
            # sum / deg.clamp(1) -- the mean reducer's own order (tensor.py:308-325)
            agg = B.gcn_aggregate(gidx, x, None, b if pre else None, n_dst,
                                  row_div=degs.clamp(min=1))
        else:
            # (sum + h_dst) / (deg + 1) (sageconv.py:131-139)
            inv = 1.0 / (degs + 1)
            xd = B.project(feat_dst, w.t()) if pre else feat_dst
            agg = B.gcn_aggregate(gidx, x, inv, b if pre else None, n_dst,
                                  addend=xd[:n_dst] * inv.view(-1, 1))
        return agg if pre else B.project(agg, w.t(), b)

    def forward(self, graph, feat):
        graph = graph.local_var()
        if isinstance(feat, tuple):
            feat_src = self.feat_drop(feat[0])
            feat_dst = self.feat_drop(feat[1])
        else:
            feat_src = feat_dst = self.feat_drop(feat)
        h_self = feat_dst
        if self._aggre_type == "gcn" and feat_src.shape[1:] != feat_dst.shape[1:]:
            raise DGLError("The feature shape of source nodes: {} should be equal to the "
                           "feature shape of destination nodes: {}.".format(
                               feat_src.shape, feat_dst.shape))
        if self._fusable(feat_src):
            rst = self._fused_neigh(graph, feat_src, feat_dst)
        else:
            if self._aggre_type == "mean":
                graph.srcdata["h"] = feat_src
                graph.update_all(fn.copy_src("h", "m"), fn.mean("m", "neigh"))
                h_neigh = graph.dstdata["neigh"]
            elif self._aggre_type == "gcn":
                graph.srcdata["h"] = feat_src
                graph.update_all(fn.copy_src("h", "m"), fn.sum("m", "neigh"))
                degs = graph.in_degrees().to(feat_dst)
                h_neigh = (graph.dstdata["neigh"] + feat_dst) / (degs.unsqueeze(-1) + 1)
            elif self._aggre_type == "pool":
                graph.srcdata["h"] = F.relu(self.fc_pool(feat_src))
                graph.update_all(fn.copy_src("h", "m"), fn.max("m", "neigh"))
                h_neigh = graph.dstdata["neigh"]
            else:
                graph.srcdata["h"] = feat_src
                graph.update_all(fn.copy_src("h", "m"), self._lstm_reducer)
                h_neigh = graph.dstdata["neigh"]
            rst = self.fc_neigh(h_neigh)
        if self._aggre_type != "gcn":
            rst = self.fc_self(h_self) + rst
        if self.activation is not None:
            rst = self.activation(rst)
        if self.norm is not None:
            rst = self.norm(rst)
        return rst
