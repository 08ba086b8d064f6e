"""``dgl.data.utils`` (``python/dgl/data/utils.py:14``): the graph serialization entry points."""
from .graph_serialize import save_graphs, load_graphs, load_labels  # noqa: F401

__all__ = ["save_graphs", "load_graphs", "load_labels"]
