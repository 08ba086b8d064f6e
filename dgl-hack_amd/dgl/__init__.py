"""MI355X-native g-SpMM / g-SDDMM engine with the DGL 0.4 operator surface.

Drop-in for the reference's message-passing hot path (ydwu4/dgl-hack):
``dgl.DGLGraph`` (update_all / apply_edges / pull / send_and_recv),
``dgl.function`` builtins, ``dgl.backend`` (``binary_reduce`` /
``copy_reduce``), ``dgl.kernel`` (the C-ABI wrappers) and
``dgl.nn.pytorch.{GraphConv, GATConv, edge_softmax}``.  Compute runs in
hand-written HIP kernels for gfx950 (``libdglmi.so``); there is no CPU path.
"""
from ._ffi import DGLError  # noqa: F401
from . import function  # noqa: F401
from . import backend  # noqa: F401
from . import kernel  # noqa: F401
from .graph import DGLGraph, ALL  # noqa: F401
from .graph_index import GraphIndex  # noqa: F401
from .heterograph import (DGLHeteroGraph, heterograph, graph, bipartite,  # noqa: F401
                          hetero_from_relations)
from .transform import (laplacian_lambda_max, add_self_loop, remove_self_loop,  # noqa: F401
                        reverse, to_bidirected, metis_partition,
                        partition_graph_with_halo)
from . import transform  # noqa: F401
from . import data  # noqa: F401
from . import nn  # noqa: F401

__version__ = "0.4"
