"""Neural-network modules (``dgl.nn``); PyTorch only."""
from . import pytorch  # noqa: F401
