"""FusedGATConv (``python/dgl/nn/pytorch/conv/fusedGatConv.py:16-166``).

GATConv whose attention softmax and aggregation run as one fused HIP kernel
(``dgl.backend.fused_gat``, csrc/kernels_gat.hip).  Falls back to the
unfused GATConv composition when the head size is not supported by the fused
kernel.  The reference's module builds ``attn_drop`` but never applies it
(fusedGatConv.py:80, 152); here it is applied in training, inside the fused
kernel (a hashed per-edge, per-head mask; ``dgl.backend.fused_gat``).  The
reference's timing prints are not reproduced.
"""

from .... import backend as B
from .gatconv import GATConv


class FusedGATConv(GATConv):
    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0., attn_drop=0.,
                 negative_slope=0.2, residual=False, activation=None):
        super(FusedGATConv, self).__init__(in_feats, out_feats, num_heads, feat_drop, attn_drop,
                                           negative_slope, residual, activation)

    def forward(self, graph, feat):
        if not self._fused_ok():
            return super(FusedGATConv, self).forward(graph, feat)
        if isinstance(feat, tuple):
            h_src = self.feat_drop(feat[0])
            h_dst = self.feat_drop(feat[1])
            feat_src = B.project(h_src, self.fc_src.weight.t()).view(-1, self._num_heads, self._out_feats)
            feat_dst = B.project(h_dst, self.fc_dst.weight.t()).view(-1, self._num_heads, self._out_feats)
        else:
            h_src = h_dst = self.feat_drop(feat)
            feat_src = feat_dst = B.project(h_src, self.fc.weight.t()).view(-1, self._num_heads, self._out_feats)
        el = (feat_src * self.attn_l).sum(dim=-1).unsqueeze(-1)
        er = (feat_dst * self.attn_r).sum(dim=-1).unsqueeze(-1)
        rst = self._fused(graph, feat_src, el, er)
        if self.res_fc is not None:
            resval = self.res_fc(h_dst).view(h_dst.shape[0], -1, self._out_feats)
            rst = rst + resval
        if self.activation:
            rst = self.activation(rst)
        return rst
