"""CFConv and ShiftedSoftplus (``python/dgl/nn/pytorch/conv/cfconv.py:9-97``).

SchNet's continuous-filter convolution: node and edge projections in torch,
then one ``u_mul_e_sum`` kernel (hv: (N, H) x he: (E, H)) and the output MLP.
"""
import numpy as np
from torch import nn

from .... import function as fn


class ShiftedSoftplus(nn.Module):
    def __init__(self, beta=1, shift=2, threshold=20):
        super(ShiftedSoftplus, self).__init__()
        self.shift = shift
        self.softplus = nn.Softplus(beta=beta, threshold=threshold)

    def forward(self, inputs):
        return self.softplus(inputs) - np.log(float(self.shift))


class CFConv(nn.Module):
    def __init__(self, node_in_feats, edge_in_feats, hidden_feats, out_feats):
        super(CFConv, self).__init__()
        self.project_edge = nn.Sequential(
            nn.Linear(edge_in_feats, hidden_feats), ShiftedSoftplus(),
            nn.Linear(hidden_feats, hidden_feats), ShiftedSoftplus())
        self.project_node = nn.Linear(node_in_feats, hidden_feats)
        self.project_out = nn.Sequential(nn.Linear(hidden_feats, out_feats), ShiftedSoftplus())

    def forward(self, g, node_feats, edge_feats):
        g = g.local_var()
        g.ndata["hv"] = self.project_node(node_feats)
        g.edata["he"] = self.project_edge(edge_feats)
        g.update_all(fn.u_mul_e("hv", "he", "m"), fn.sum("m", "h"))
        return self.project_out(g.ndata["h"])
