"""Graph convolution modules."""
from .graphconv import GraphConv  # noqa: F401
from .gatconv import GATConv  # noqa: F401
from .fused_gatconv import FusedGATConv  # noqa: F401
from .relgraphconv import RelGraphConv  # noqa: F401
