"""``dgl.data`` (``python/dgl/data/__init__.py``): the graph file format only -- the dataset
downloaders need network access and sit outside the hot path's scope."""
from .utils import *  # noqa: F401,F403
