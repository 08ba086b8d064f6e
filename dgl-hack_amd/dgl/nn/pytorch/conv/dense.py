"""Dense-adjacency conv modules (``python/dgl/nn/pytorch/conv/densegraphconv.py``,
``densesageconv.py``, ``densechebconv.py``).

They take a dense (N_dst x N_src) adjacency instead of a graph: the
aggregation is a dense GEMM (hipBLASLt on MFMA), not the sparse kernels, and
they exist so code written against the reference finds them.  Same
parameters, initialisation and math as the reference; ``DenseChebConv``
computes lambda_max with ``torch.linalg.eigvals`` (the reference's
``torch.eig`` is gone from current PyTorch).
"""
import torch as th
from torch import nn
from torch.nn import init

from ...._ffi import DGLError


class DenseGraphConv(nn.Module):
    def __init__(self, in_feats, out_feats, norm="both", bias=True, activation=None):
        super(DenseGraphConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._norm = norm
        self.weight = nn.Parameter(th.Tensor(in_feats, out_feats))
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_buffer("bias", None)
        self.reset_parameters()
        self._activation = activation

    def reset_parameters(self):
        init.xavier_uniform_(self.weight)
        if self.bias is not None:
            init.zeros_(self.bias)

    def forward(self, adj, feat):
        adj = adj.float().to(feat.device)
        shp = (1,) * (feat.dim() - 1)
        if self._norm == "both":
            nsrc = adj.sum(dim=0).clamp(min=1).pow(-0.5)
            feat = feat * nsrc.reshape(nsrc.shape + shp)
        if self._in_feats > self._out_feats:
            rst = adj @ th.matmul(feat, self.weight)
        else:
            rst = th.matmul(adj @ feat, self.weight)
        if self._norm != "none":
            deg = adj.sum(dim=1).clamp(min=1)
            ndst = deg.pow(-0.5) if self._norm == "both" else 1.0 / deg
            rst = rst * ndst.reshape(ndst.shape + shp)
        if self.bias is not None:
            rst = rst + self.bias
        if self._activation is not None:
            rst = self._activation(rst)
        return rst


class DenseSAGEConv(nn.Module):
    """The 'gcn' aggregator of SAGEConv on a dense adjacency."""

    def __init__(self, in_feats, out_feats, feat_drop=0., bias=True, norm=None, activation=None):
        super(DenseSAGEConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._norm = norm
        self.feat_drop = nn.Dropout(feat_drop)
        self.activation = activation
        self.fc = nn.Linear(in_feats, out_feats, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.fc.weight, gain=nn.init.calculate_gain("relu"))

    def forward(self, adj, feat):
        if isinstance(feat, tuple):
            if feat[0].shape[1:] != feat[1].shape[1:]:
                raise DGLError("The feature shape of source nodes: {} should be equal to the "
                               "feature shape of destination nodes: {}.".format(
                                   feat[0].shape, feat[1].shape))
            feat_src, feat_dst = self.feat_drop(feat[0]), self.feat_drop(feat[1])
        else:
            feat_src = feat_dst = self.feat_drop(feat)
        adj = adj.float().to(feat_src.device)
        deg = adj.sum(dim=1, keepdim=True)
        rst = self.fc((adj @ feat_src + feat_dst) / (deg + 1))
        if self.activation is not None:
            rst = self.activation(rst)
        if self._norm is not None:
            rst = self._norm(rst)
        return rst


class DenseChebConv(nn.Module):
    def __init__(self, in_feats, out_feats, k, bias=True):
        super(DenseChebConv, self).__init__()
        self._in_feats = in_feats
        self._out_feats = out_feats
        self._k = k
        self.W = nn.Parameter(th.Tensor(k, in_feats, out_feats))
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_buffer("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.bias is not None:
            init.zeros_(self.bias)
        for i in range(self._k):
            init.xavier_normal_(self.W[i], init.calculate_gain("relu"))

    def forward(self, adj, feat, lambda_max=None):
        A = adj.to(feat)
        n = A.shape[0]
        dinv = A.sum(dim=1).clamp(min=1).pow(-0.5)
        eye = th.eye(n, dtype=A.dtype, device=A.device)
        L = eye - dinv[:, None] * A * dinv[None, :]
        if lambda_max is None:
            # the reference's th.eig takes every eigenvalue of a general matrix; a
            # symmetric adjacency (undirected graph) gives a symmetric L, whose
            # spectrum eigvalsh finds far faster (pass lambda_max, e.g. from
            # dgl.laplacian_lambda_max, to skip the decomposition altogether)
            if th.equal(A, A.transpose(0, 1)):
                lambda_max = th.linalg.eigvalsh(L).max()
            else:
                lambda_max = th.linalg.eigvals(L).real.max()
        L_hat = 2 * L / lambda_max - eye
        Z = [eye]
        for i in range(1, self._k):
            Z.append(L_hat if i == 1 else 2 * L_hat @ Z[-1] - Z[-2])
        rst = (th.stack(Z, 0) @ feat.unsqueeze(0) @ self.W).sum(0)
        if self.bias is not None:
            rst = rst + self.bias
        return rst
