"""FusedGATConv (``python/dgl/nn/pytorch/conv/fusedGatConv.py:16-166``).

GATConv whose attention softmax and aggregation run as one fused HIP kernel
(``dgl.backend.fused_gat``, csrc/kernels_gat.hip).  Falls back to the
unfused GATConv composition when the head size is not supported by the fused
kernel.  The reference's module builds ``attn_drop`` but never applies it
(fusedGatConv.py:80, 152); here it is applied in training, inside the fused
kernel (a hashed per-edge, per-head mask; ``dgl.backend.fused_gat``).  The
forward is GATConv's, which takes the fused kernels whenever they apply
(``GATConv._fused_route``).  The reference's timing prints are not reproduced.
"""

from .gatconv import GATConv


class FusedGATConv(GATConv):
    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0., attn_drop=0.,
                 negative_slope=0.2, residual=False, activation=None):
        super(FusedGATConv, self).__init__(in_feats, out_feats, num_heads, feat_drop, attn_drop,
                                           negative_slope, residual, activation)
