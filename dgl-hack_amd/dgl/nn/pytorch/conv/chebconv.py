"""ChebConv (``python/dgl/nn/pytorch/conv/chebconv.py:12-127``).

Chebyshev polynomials of the scaled Laplacian:  T0 = X,
T1 = -2/lambda * A X + (2/lambda - 1) X,
Tk = -4/lambda * A T(k-1) + (4/lambda - 2) T(k-1) - T(k-2)
(A = D^-1/2 A D^-1/2, in-degree norm on both sides as the reference).  Each
polynomial term is ONE copy_u_sum launch: the destination norm times the
-2/lambda (-4/lambda) factor and the recurrence's other terms run in the
kernel's epilogue (row_mul + addend, ``dgl.backend.gcn_aggregate``).
``lambda_max`` defaults to ``dgl.laplacian_lambda_max(graph)`` (host scipy,
as the reference; pass it explicitly to keep the forward on the device).
"""
import torch as th
from torch import nn
from torch.nn import init

from .... import backend as B
from .... import function as fn
from ....transform import laplacian_lambda_max
from .sgconv import in_degree_norm


class ChebConv(nn.Module):
    def __init__(self, in_feats, out_feats, k, bias=True):
        super(ChebConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self.fc = nn.ModuleList([nn.Linear(in_feats, out_feats, bias=False) for _ in range(k)])
        self._k = k
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_buffer("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.bias is not None:
            init.zeros_(self.bias)
        for module in self.fc.modules():
            if isinstance(module, nn.Linear):
                init.xavier_normal_(module.weight, init.calculate_gain("relu"))
                if module.bias is not None:
                    init.zeros_(module.bias)

    def forward(self, graph, feat, lambda_max=None):
        graph = graph.local_var()
        n = graph.number_of_nodes()
        norm = in_degree_norm(graph, feat.device)
        if lambda_max is None:
            lambda_max = laplacian_lambda_max(graph)
        lam = th.as_tensor(lambda_max, dtype=th.float32, device=feat.device).reshape(-1)
        if lam.numel() == 1:
            lam = lam.expand(n)
        elif lam.numel() != n:
            raise ValueError("lambda_max must hold one value (one graph) or one per node")
        lam = lam.contiguous()
        fused = (getattr(self, "fused", True) and feat.dim() == 2
                 and feat.dtype == th.float32 and feat.is_cuda)
        gidx = graph._graph.get_immutable_gidx(feat.device) if fused else None

        def hop(x, coef, addend):
            # coef * (norm * A (norm * x)) + addend
            if fused:
                return B.gcn_aggregate(gidx, x * norm.view(-1, 1), norm * coef, None, n,
                                       addend=addend)
            graph.ndata["h"] = x * norm.view(-1, 1)
            graph.update_all(fn.copy_u("h", "m"), fn.sum("m", "h"))
            return graph.ndata.pop("h") * norm.view(-1, 1) * coef.view(-1, 1) + addend

        lam_c = lam.view(-1, 1)
        tx_0 = feat
        rst = self.fc[0](tx_0)
        if self._k > 1:
            tx_1 = hop(tx_0, -2.0 / lam, tx_0 * (2.0 / lam_c - 1))
            rst = rst + self.fc[1](tx_1)
        for i in range(2, self._k):
            tx_2 = hop(tx_1, -4.0 / lam, tx_1 * (4.0 / lam_c - 2) - tx_0)
            rst = rst + self.fc[i](tx_2)
            tx_1, tx_0 = tx_2, tx_1
        if self.bias is not None:
            rst = rst + self.bias
        return rst
