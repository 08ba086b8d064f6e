"""FusedGATConv (``python/dgl/nn/pytorch/conv/fusedGatConv.py:16-166``).

GATConv whose attention softmax and aggregation run as one fused HIP kernel
(``dgl.backend.fused_gat``, csrc/kernels_gat.hip).  Falls back to the
unfused GATConv composition when the head size is not supported by the fused
kernel.  As in the reference, ``attn_drop`` is built but never applied
(fusedGatConv.py:80 builds it, :152 calls ``B.fused_gat`` without it): training and
eval outputs are the same.  The forward is GATConv's, which takes the fused kernels
whenever they apply (``GATConv._fused_route``).  The reference's timing prints and
``th.cuda.synchronize()`` calls are not reproduced.
"""

from .gatconv import GATConv


class FusedGATConv(GATConv):
    _applies_attn_drop = False

    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0., attn_drop=0.,
                 negative_slope=0.2, residual=False, activation=None):
        super(FusedGATConv, self).__init__(in_feats, out_feats, num_heads, feat_drop, attn_drop,
                                           negative_slope, residual, activation)
