"""PyTorch modules (``dgl.nn.pytorch``)."""
from .conv import GraphConv, GATConv, FusedGATConv, RelGraphConv  # noqa: F401
from .softmax import edge_softmax  # noqa: F401
from .hetero import HeteroGraphConv  # noqa: F401
