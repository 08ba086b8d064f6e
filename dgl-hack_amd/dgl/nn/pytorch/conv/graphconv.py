"""GraphConv (``python/dgl/nn/pytorch/conv/graphconv.py:11-188``).

Same parameters, initialisation and computation order as the reference:
``norm`` in {'none','both','right'}; the dense projection (a torch GEMM on
MFMA through hipBLASLt) goes before the aggregation when in_feats >
out_feats, after it otherwise; the aggregation is one ``copy_u_sum`` on the
load-balanced HIP kernel.

On 2-D float32 features the destination-side norm and the bias are fused into
that aggregation kernel's epilogue (``dgl.backend.gcn_aggregate``): for
in_feats > out_feats ``out = (A X W) * norm + bias`` in one launch; otherwise
``(A X) * norm`` in the launch and the bias inside the projection GEMM
(``project(..., bias)``, hipBLASLt addmm) -- the row scaling commutes with the
right-multiplication by W.  ``fused = False`` on the module restores the
reference's separate steps.

With ``norm`` 'both' or 'right' on a whole graph, both norms become one constant
weight per edge streamed in the kernel's walk order (``dgl.backend
.gcn_norm_aggregate``): the forward and the gradient of the features are one
launch each, without the three elementwise (N, F) passes of the source-side
scaling, its gradient and the scaled incoming gradient.
"""
import torch as th
from torch import nn
from torch.nn import init

from .... import backend as B
from .... import function as fn
from ...._ffi import DGLError


class GraphConv(nn.Module):
    def __init__(self, in_feats, out_feats, norm="both", weight=True, bias=True,
                 activation=None):
        super(GraphConv, self).__init__()
        if norm not in ("none", "both", "right"):
            raise DGLError('Invalid norm value. Must be either "none", "both" or "right".'
                           ' But got "{}".'.format(norm))
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._norm = norm
        if weight:
            self.weight = nn.Parameter(th.Tensor(in_feats, out_feats))
        else:
            self.register_parameter("weight", None)
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()
        self._activation = activation

    def reset_parameters(self):
        if self.weight is not None:
            init.xavier_uniform_(self.weight)
        if self.bias is not None:
            init.zeros_(self.bias)

    def forward(self, graph, feat, weight=None):
        graph = graph.local_var()
        if weight is not None:
            if self.weight is not None:
                raise DGLError("External weight is provided while at the same time the"
                               " module has defined its own weight parameter. Please"
                               " create the module with flag weight=False.")
        else:
            weight = self.weight
        if self._norm != "none" and self._edge_weight_path(graph, feat):
            return self._edge_weight_forward(graph, feat, weight)
        if self._norm == "both":
            degs = graph._device_degrees(feat.device, "out").float().clamp(min=1)
            norm = th.pow(degs, -0.5)
            norm = th.reshape(norm, norm.shape + (1,) * (feat.dim() - 1))
            feat = feat * norm
        if getattr(self, "fused", True) and feat.dim() == 2 and feat.dtype == th.float32:
            rst = self._fused_forward(graph, feat, weight)
        else:
            rst = self._reference_forward(graph, feat, weight)
        if self._activation is not None:
            rst = self._activation(rst)
        return rst

    def _edge_weight_path(self, graph, feat):
        """Both norms as one streamed per-edge weight (dgl.backend
        .gcn_norm_aggregate): whole graphs whose aggregation runs as one pass (no
        column blocks, which only the unweighted copy_u sum takes)."""
        if not getattr(self, "fused", True) or feat.dim() != 2 or feat.dtype != th.float32:
            return False
        if not hasattr(graph._graph, "get_immutable_gidx") or not feat.is_cuda:
            return False
        gidx = graph._graph.get_immutable_gidx(feat.device)
        f = self._out_feats if self._in_feats > self._out_feats else self._in_feats
        from .... import kernel as K
        return bool(gidx.eid_perm) and K.spmm_col_blocks(gidx, f) == 1

    def _edge_weight_forward(self, graph, feat, weight):
        gidx = graph._graph.get_immutable_gidx(feat.device)
        n_dst = graph.number_of_dst_nodes()
        if self._in_feats > self._out_feats:
            if weight is not None:
                feat = B.project(feat, weight)
            rst = B.gcn_norm_aggregate(gidx, feat, self._norm, self.bias, n_dst)
        else:
            rst = B.gcn_norm_aggregate(gidx, feat, self._norm, None, n_dst)
            if weight is not None:
                rst = B.project(rst, weight, self.bias)
            elif self.bias is not None:
                rst = rst + self.bias
        if self._activation is not None:
            rst = self._activation(rst)
        return rst

    def _dst_norm(self, graph, device):
        if self._norm == "none":
            return None
        degs = graph._device_degrees(device, "in").float().clamp(min=1)
        return th.pow(degs, -0.5) if self._norm == "both" else 1.0 / degs

    def _fused_forward(self, graph, feat, weight):
        gidx = graph._graph.get_immutable_gidx(feat.device)
        n_dst = graph.number_of_dst_nodes()
        norm = self._dst_norm(graph, feat.device)
        if self._in_feats > self._out_feats:
            if weight is not None:
                feat = B.project(feat, weight)
            return B.gcn_aggregate(gidx, feat, norm, self.bias, n_dst)
        rst = B.gcn_aggregate(gidx, feat, norm, None, n_dst)
        if weight is not None:
            return B.project(rst, weight, self.bias)
        return rst if self.bias is None else rst + self.bias

    def _reference_forward(self, graph, feat, weight):
        if self._in_feats > self._out_feats:
            if weight is not None:
                feat = B.project(feat, weight)
            graph.srcdata["h"] = feat
            graph.update_all(fn.copy_src(src="h", out="m"), fn.sum(msg="m", out="h"))
            rst = graph.dstdata["h"]
        else:
            graph.srcdata["h"] = feat
            graph.update_all(fn.copy_src(src="h", out="m"), fn.sum(msg="m", out="h"))
            rst = graph.dstdata["h"]
            if weight is not None:
                rst = B.project(rst, weight)
        if self._norm != "none":
            norm = self._dst_norm(graph, feat.device)
            rst = rst * th.reshape(norm, norm.shape + (1,) * (feat.dim() - 1))
        if self.bias is not None:
            rst = rst + self.bias
        return rst

    def extra_repr(self):
        summary = "in={_in_feats}, out={_out_feats}, normalization={_norm}"
        if "_activation" in self.__dict__:
            summary += ", activation={_activation}"
        return summary.format(**self.__dict__)
