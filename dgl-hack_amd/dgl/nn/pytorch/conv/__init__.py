"""Graph convolution modules."""
from .graphconv import GraphConv  # noqa: F401
from .gatconv import GATConv  # noqa: F401
