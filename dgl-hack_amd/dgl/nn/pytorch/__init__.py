"""PyTorch modules (``dgl.nn.pytorch``)."""
from .conv import (GraphConv, GATConv, FusedGATConv, RelGraphConv, SAGEConv,  # noqa: F401
                   GINConv, SGConv, APPNPConv, TAGConv, ChebConv, AGNNConv, EdgeConv,
                   GatedGraphConv, DenseGraphConv,
                   DenseSAGEConv, DenseChebConv)
from .softmax import edge_softmax  # noqa: F401
from .hetero import HeteroGraphConv  # noqa: F401
