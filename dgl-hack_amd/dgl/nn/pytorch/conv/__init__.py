"""Graph convolution modules (``python/dgl/nn/pytorch/conv/__init__.py``)."""
from .graphconv import GraphConv  # noqa: F401
from .gatconv import GATConv  # noqa: F401
from .fused_gatconv import FusedGATConv  # noqa: F401
from .relgraphconv import RelGraphConv  # noqa: F401
from .sageconv import SAGEConv  # noqa: F401
from .ginconv import GINConv  # noqa: F401
from .sgconv import SGConv  # noqa: F401
from .appnpconv import APPNPConv  # noqa: F401
from .tagconv import TAGConv  # noqa: F401
from .chebconv import ChebConv  # noqa: F401
from .agnnconv import AGNNConv  # noqa: F401
from .edgeconv import EdgeConv  # noqa: F401
from .gatedgraphconv import GatedGraphConv  # noqa: F401
from .dense import DenseGraphConv, DenseSAGEConv, DenseChebConv  # noqa: F401
