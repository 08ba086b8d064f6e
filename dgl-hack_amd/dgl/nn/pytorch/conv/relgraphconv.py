"""RelGraphConv (``python/dgl/nn/pytorch/conv/relgraphconv.py``).

Same parameters, regularisers ("basis", "bdd"), initialisation and forward
signature ``forward(g, x, etypes, norm=None)`` as the reference, whose message
function is a per-edge batched matmul UDF (``bmm_maybe_select``).  Here the
relation transforms are dense GEMMs over the node features (one per relation,
on MFMA) and all relations are aggregated by one typed gather kernel
(``dgl.backend.rgcn_layer1``): per edge the bytes of one output row instead of
an F_in x F_out product.  Layers whose gathered rows are 64 floats both ways
(64 -> 64, up to 4 relations) with a constant norm instead run the hack's fused
layer-1 C entries (aggregate per relation, then transform, in one kernel; DESIGN.md
4.4).
"""
import torch as th
from torch import nn

from .... import backend as B


class RelGraphConv(nn.Module):
    def __init__(self, in_feat, out_feat, num_rels, regularizer="basis", num_bases=None,
                 bias=True, activation=None, self_loop=False, dropout=0.0):
        super(RelGraphConv, self).__init__()
        self.in_feat = in_feat
        self.out_feat = out_feat
        self.num_rels = num_rels
        self.regularizer = regularizer
        self.num_bases = num_bases
        if self.num_bases is None or self.num_bases > self.num_rels or self.num_bases <= 0:
            self.num_bases = self.num_rels
        self.bias = bias
        self.activation = activation
        self.self_loop = self_loop
        if regularizer == "basis":
            self.weight = nn.Parameter(th.Tensor(self.num_bases, self.in_feat, self.out_feat))
            if self.num_bases < self.num_rels:
                self.w_comp = nn.Parameter(th.Tensor(self.num_rels, self.num_bases))
            nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain("relu"))
            if self.num_bases < self.num_rels:
                nn.init.xavier_uniform_(self.w_comp, gain=nn.init.calculate_gain("relu"))
        elif regularizer == "bdd":
            if in_feat % self.num_bases != 0 or out_feat % self.num_bases != 0:
                raise ValueError("Feature size must be a multiplier of num_bases (%d)."
                                 % self.num_bases)
            self.submat_in = in_feat // self.num_bases
            self.submat_out = out_feat // self.num_bases
            self.weight = nn.Parameter(th.Tensor(
                self.num_rels, self.num_bases * self.submat_in * self.submat_out))
            nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain("relu"))
        else:
            raise ValueError("Regularizer must be either 'basis' or 'bdd'")
        if self.bias:
            self.h_bias = nn.Parameter(th.Tensor(out_feat))
            nn.init.zeros_(self.h_bias)
        if self.self_loop:
            self.loop_weight = nn.Parameter(th.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
        self.dropout = nn.Dropout(dropout)
        # extension: layers of 64-float rows (both ways) with a constant norm run on the
        # fused layer-1 kernels (dgl.backend.rgcn_fused_route); False keeps the
        # GEMM + typed-gather path below
        self.use_fused = True

    def _relation_weights(self):
        if self.num_bases < self.num_rels:
            w = self.weight.view(self.num_bases, self.in_feat * self.out_feat)
            return th.matmul(self.w_comp, w).view(self.num_rels, self.in_feat, self.out_feat)
        return self.weight

    def _transform(self, x):
        """Y = x_u W_r for every (node, relation), as rows of the typed gather.

        Returns (y, node_major): one-hot input gives the (R, N, out) slice of the
        weights (relation-major rows); feature input gives ONE GEMM
        X [W_0 | ... | W_{R-1}] of shape (N, R * out) (node-major rows) -- not R
        broadcast GEMMs over an expanded copy of X."""
        if x.dtype == th.int64 and x.dim() == 1:
            if self.regularizer == "bdd":
                raise TypeError("Block decomposition does not allow integer ID feature.")
            return self._relation_weights()[:, x, :], False   # one-hot input (layer 0)
        R, fo = self.num_rels, self.out_feat
        if self.regularizer == "basis":
            w = self._relation_weights().permute(1, 0, 2).reshape(self.in_feat, R * fo)
            return B.project(x, w), True
        w = self.weight.view(R, self.num_bases, self.submat_in, self.submat_out)
        xb = x.view(x.shape[0], self.num_bases, self.submat_in)
        return th.einsum("nbi,rbio->nrbo", xb, w), True

    def forward(self, g, x, etypes, norm=None):
        if self.use_fused and self.regularizer == "basis":
            route = B.rgcn_fused_route(g, x, (self.num_rels, self.in_feat, self.out_feat), norm,
                                       etypes, self.self_loop)
            if route is not None:
                # aggregate-then-transform on the fused layer-1 C entries, the self-loop
                # message and the bias in the same kernel (B.rgcn_fused_layer1)
                node_repr = B.rgcn_fused_layer1(route, x, self._relation_weights(),
                                                self.loop_weight if self.self_loop else None,
                                                self.h_bias if self.bias else None)
                if self.activation:
                    node_repr = self.activation(node_repr)
                return self.dropout(node_repr)
        y, node_major = self._transform(x)
        y = y.contiguous()
        n = g.number_of_nodes()
        loop = None
        if self.self_loop:
            loop = self.loop_weight[x] if (x.dtype == th.int64 and x.dim() == 1) else \
                B.project(x, self.loop_weight)
        # bias and self-loop term fused into the aggregation's epilogue when the norm
        # is constant (node_repr = agg + h_bias + loop, as relgraphconv.py:150-160)
        node_repr = B._typed_aggregate(g, self.num_rels, y.view(self.num_rels * n, self.out_feat),
                                       norm, etypes, node_major,
                                       bias=self.h_bias if self.bias else None,
                                       addend=loop.contiguous() if loop is not None else None)
        if self.activation:
            node_repr = self.activation(node_repr)
        return self.dropout(node_repr)
