"""DGLGraph: the drop-in graph object for the g-SpMM / g-SDDMM path.

A thin, reference-compatible subset of ``python/dgl/graph.py``: node / edge
storage with ``ndata`` / ``edata`` (and the ``srcdata`` / ``dstdata``
aliases of a homogeneous graph), ``local_var``, degree queries, and the
message-passing entry points whose builtin forms lower to one kernel each:

* ``update_all(msg, reduce)``        -> ``F.copy_reduce`` / ``F.binary_reduce``
  (``graph.py:3221-3264``, ``runtime/scheduler.py:196-252, 905-917``);
* ``pull(v, msg, reduce)`` / ``send_and_recv(edges, msg, reduce)`` / ``push(u, ...)``
  -> the same kernels on the in-edge subgraph (``scheduler.py:154-194, 254-332,
  417-449``);
* ``send(edges, msg)`` + ``recv(v, reduce)`` -> messages materialised per edge
  (reducer ``"none"``), then ``copy_e`` reduced over the pending edges
  (``scheduler.py:31-129``);
* ``apply_edges(msg)``              -> reducer ``"none"`` (``graph.py:2600``,
  ``scheduler.py:334-375``).

Functions registered with ``register_{message,reduce,apply_node,apply_edge}_func``
are the defaults of every entry point.  User-defined message functions are
materialised per edge and reduced by a builtin reducer as ``copy_e`` (what the
reference's scheduler does, ``scheduler.py:919-960``); ``apply_edges`` /
``apply_nodes`` accept UDFs (plain tensor gathers).  A user-defined *reduce*
runs the reference's degree bucketing on the device (messages materialised per
edge, one UDF call per in-degree bucket on a (nodes, degree, ...) mailbox,
``runtime/degree_bucketing.py``, ``src/scheduler/scheduler.cc``): torch tensor
ops, off the kernel path, as in the reference.
"""
from __future__ import annotations

from collections.abc import MutableMapping

import numpy as np
import torch as th

from . import backend as B
from ._ffi import DGLError
from .function.base import TargetCode
from .function.message import MessageFunction
from .function.reducer import ReduceFunction
from .graph_index import GraphIndex
from .init import zero_initializer

ALL = "__ALL__"


def is_all(x):
    return isinstance(x, str) and x == ALL


def _to_index_array(x, name):
    if isinstance(x, th.Tensor):
        return x.detach().to("cpu", th.int64).numpy().reshape(-1)
    return np.asarray(x, dtype=np.int64).reshape(-1)


class Frame(MutableMapping):
    """Columns of per-node or per-edge features (``python/dgl/frame.py``), with the
    per-column initializers of ``frame.py:219-260`` (default: zeros)."""

    def __init__(self, num_rows_fn, data=None, initializers=None):
        self._num_rows = num_rows_fn
        self._cols = dict(data) if data else {}
        self._inits = dict(initializers) if initializers else {}

    def set_initializer(self, initializer, column=None):
        self._inits[column] = initializer

    def get_initializer(self, column=None):
        return self._inits.get(column, self._inits.get(None, zero_initializer))

    def init_rows(self, column, like, ids):
        """Rows ``ids`` (a device id tensor) of ``column`` from its initializer, shaped
        and typed like ``like`` (a tensor with the column's row shape)."""
        shape = (int(ids.shape[0]),) + tuple(like.shape[1:])
        return self.get_initializer(column)(shape, like.dtype, like.device, ids)

    def __getitem__(self, key):
        return self._cols[key]

    def __setitem__(self, key, val):
        if not isinstance(val, th.Tensor):
            raise DGLError("Feature %s must be a torch tensor" % key)
        n = self._num_rows()
        if val.dim() == 0 or val.shape[0] != n:
            raise DGLError("Expected feature %s with first dimension %d, got shape %s"
                           % (key, n, tuple(val.shape)))
        self._cols[key] = val

    def __delitem__(self, key):
        del self._cols[key]

    def __iter__(self):
        return iter(self._cols)

    def __len__(self):
        return len(self._cols)

    def __repr__(self):
        return repr({k: tuple(v.shape) for k, v in self._cols.items()})

    def clone(self):
        return Frame(self._num_rows, self._cols, self._inits)


class EdgeBatch(object):
    """Edges given to a message UDF (``python/dgl/udf.py:EdgeBatch``)."""

    def __init__(self, src, dst, eid, src_data, dst_data, edge_data):
        self._src, self._dst, self._eid = src, dst, eid
        self.src = src_data
        self.dst = dst_data
        self.data = edge_data

    def edges(self):
        return self._src, self._dst, self._eid

    def batch_size(self):
        return int(self._eid.shape[0])

    def __len__(self):
        return self.batch_size()


class NodeBatch(object):
    """Nodes given to an apply or reduce UDF (``python/dgl/udf.py:NodeBatch``);
    ``mailbox`` holds a reduce UDF's messages, (nodes, degree, ...) per field."""

    def __init__(self, nodes, data, mailbox=None):
        self._nodes = nodes
        self.data = data
        self.mailbox = mailbox

    def nodes(self):
        return self._nodes

    def batch_size(self):
        return int(self._nodes.shape[0])

    def __len__(self):
        return self.batch_size()


class _Space(object):
    __slots__ = ["data"]

    def __init__(self, data):
        self.data = data


class _RowView(MutableMapping):
    """``G.nodes[ids].data`` / ``G.edges[ids].data`` (view.py:46-81, 114-150)."""

    def __init__(self, graph, sel, node):
        self._g, self._sel, self._node = graph, sel, node

    def _frame(self):
        return self._g._node_frame if self._node else self._g._edge_frame

    def __getitem__(self, key):
        get = self._g.get_n_repr if self._node else self._g.get_e_repr
        return get(self._sel)[key]

    def __setitem__(self, key, val):
        put = self._g.set_n_repr if self._node else self._g.set_e_repr
        put({key: val}, self._sel)

    def __delitem__(self, key):
        if not is_all(self._sel):
            raise DGLError("Delete feature data is not supported on only a subset of rows")
        del self._frame()[key]

    def __iter__(self):
        return iter(self._frame())

    def __len__(self):
        return len(self._frame())


class NodeView(object):
    """``G.nodes`` (view.py:15-44): call for all node ids, index for row data."""

    def __init__(self, graph):
        self._g = graph

    def __len__(self):
        return self._g.number_of_nodes()

    def __getitem__(self, nodes):
        if isinstance(nodes, slice):
            if not (nodes.start is None and nodes.stop is None and nodes.step is None):
                raise DGLError('Currently only full slice ":" is supported')
            return _Space(_RowView(self._g, ALL, True))
        return _Space(_RowView(self._g, nodes, True))

    def __call__(self):
        return th.arange(self._g.number_of_nodes(), dtype=th.int64)


class EdgeView(object):
    """``G.edges`` (view.py:83-112): call for the edge list, index (edge ids or a
    (u, v) pair of id lists) for row data."""

    def __init__(self, graph):
        self._g = graph

    def __len__(self):
        return self._g.number_of_edges()

    def __getitem__(self, edges):
        if isinstance(edges, slice):
            if not (edges.start is None and edges.stop is None and edges.step is None):
                raise DGLError('Currently only full slice ":" is supported')
            return _Space(_RowView(self._g, ALL, False))
        return _Space(_RowView(self._g, edges, False))

    def __call__(self, *args, **kwargs):
        return self._g.all_edges(*args, **kwargs)


class DGLGraph(object):
    """Base graph class (``python/dgl/graph.py:DGLGraph``, homogeneous)."""

    def __init__(self, graph_data=None, node_frame=None, edge_frame=None, multigraph=None,
                 readonly=False):
        self._graph = GraphIndex(0)
        self._readonly = False
        self._node_frame = Frame(self.number_of_nodes)
        self._edge_frame = Frame(self.number_of_edges)
        if graph_data is not None:
            self._init_from(graph_data)
        if node_frame is not None:
            for k, v in node_frame.items():
                self._node_frame[k] = v
        if edge_frame is not None:
            for k, v in edge_frame.items():
                self._edge_frame[k] = v
        self._readonly = bool(readonly)

    def _init_from(self, data):
        if isinstance(data, GraphIndex):
            self._graph = data
            return
        if isinstance(data, DGLGraph):
            src, dst, _ = data._graph.edges()
            self._graph.add_nodes(data.number_of_nodes())
            self._graph.add_edges(src, dst)
            return
        try:
            import networkx as nx
        except ImportError:  # pragma: no cover
            nx = None
        if nx is not None and isinstance(data, nx.Graph):
            self.from_networkx(data)
            return
        try:
            import scipy.sparse as sp
            if sp.issparse(data):
                self.from_scipy_sparse_matrix(data)
                return
        except ImportError:  # pragma: no cover
            pass
        if isinstance(data, (tuple, list)) and len(data) == 2:
            src = _to_index_array(data[0], "src")
            dst = _to_index_array(data[1], "dst")
            n = int(max(src.max(initial=-1), dst.max(initial=-1)) + 1)
            self._graph.add_nodes(n)
            self._graph.add_edges(src, dst)
            return
        raise DGLError("Unsupported graph data type: %s" % type(data))

    @classmethod
    def from_device_coo(cls, src, dst, num_nodes):
        """Read-only graph from device int32 (src, dst) tensors; CSRs built on the GPU."""
        g = cls()
        g._graph = GraphIndex.from_device_coo(src, dst, num_nodes)
        g._readonly = True
        return g

    # ---- conversion (graph_index.py:1078-1135, :1138-1163) -------------------------
    def from_networkx(self, nx_graph):
        import networkx as nx
        if self.number_of_nodes() or self.number_of_edges():
            self.clear()
        if not nx_graph.is_directed():
            nx_graph = nx_graph.to_directed()
        n = nx_graph.number_of_nodes()
        m = nx_graph.number_of_edges()
        has_id = m > 0 and "id" in next(iter(nx_graph.edges(data=True)))[-1]
        if has_id:
            src = np.zeros(m, np.int64)
            dst = np.zeros(m, np.int64)
            for u, v, attr in nx_graph.edges(data=True):
                src[attr["id"]] = u
                dst[attr["id"]] = v
        else:
            es = list(nx_graph.edges)
            src = np.array([e[0] for e in es], np.int64)
            dst = np.array([e[1] for e in es], np.int64)
        self._graph.add_nodes(n)
        self._graph.add_edges(src, dst)

    def from_scipy_sparse_matrix(self, spmat):
        """Replace the graph by ``spmat``'s edges in COO order (graph.py:1870-1901:
        clear, then build)."""
        if self.number_of_nodes() or self.number_of_edges():
            self.clear()
        coo = spmat.tocoo()
        self._graph.add_nodes(coo.shape[0])
        self._graph.add_edges(coo.row.astype(np.int64), coo.col.astype(np.int64))

    # ---- mutation ---------------------------------------------------------------
    def _check_mutable(self):
        if self._readonly:
            raise DGLError("Mutation is not allowed in read-only graph.")

    def add_nodes(self, num, data=None):
        self._check_mutable()
        old = self.number_of_nodes()
        self._graph.add_nodes(num)
        self._extend_frame(self._node_frame, old, int(num), data)

    def add_edge(self, u, v, data=None):
        self.add_edges([u], [v], data)

    def add_edges(self, u, v, data=None):
        self._check_mutable()
        old = self.number_of_edges()
        self._graph.add_edges(_to_index_array(u, "u"), _to_index_array(v, "v"))
        self._extend_frame(self._edge_frame, old, self.number_of_edges() - old, data)
        self._extend_messages(old)

    def _extend_messages(self, old):
        """New edges carry no pending message; earlier pending ones stay
        (graph.py:1044-1047, msg_index.append_zeros / msg_frame.add_rows)."""
        m = self.number_of_edges()
        ind = getattr(self, "_msg_ind", None)
        if ind is not None and ind.shape[0] == old:
            self._msg_ind = np.concatenate([ind, np.zeros(m - old, bool)])
        for k, t in (getattr(self, "_msg_frame", None) or {}).items():
            if t.shape[0] == old:
                self._msg_frame[k] = th.cat([t, t.new_zeros((m - old,) + tuple(t.shape[1:]))])

    def add_edges_with_type(self, u, v, etypes, data=None):
        """Add typed edges (the hack's graph.py:1229); types feed R-GCN kernels."""
        self._check_mutable()
        old = self.number_of_edges()
        self._graph.add_edges_with_type(_to_index_array(u, "u"), _to_index_array(v, "v"),
                                        _to_index_array(etypes, "etypes"))
        self._extend_frame(self._edge_frame, old, self.number_of_edges() - old, data)
        self._extend_messages(old)

    @staticmethod
    def _extend_frame(frame, old, num, data):
        for k in list(frame._cols.keys()):
            col = frame._cols[k]
            if data is not None and k in data:
                ext = data[k]
            else:
                ext = frame.init_rows(k, col, th.arange(old, old + num, device=col.device))
            frame._cols[k] = th.cat([col, ext.to(col.device, col.dtype)], 0)
        if data is not None:
            for k, v in data.items():
                if k not in frame._cols:
                    if old != 0:
                        raise DGLError("Cannot add new feature %s to a non-empty frame" % k)
                    frame._cols[k] = v

    # ---- queries ----------------------------------------------------------------
    def number_of_nodes(self):
        return self._graph.number_of_nodes()

    def number_of_src_nodes(self):
        return self.number_of_nodes()

    def number_of_dst_nodes(self):
        return self.number_of_nodes()

    def number_of_edges(self):
        return self._graph.number_of_edges()

    def __len__(self):
        return self.number_of_nodes()

    @property
    def is_homograph(self):
        return True

    def reverse(self, share_ndata=False, share_edata=False):
        """``graph.py`` DGLGraph.reverse -> ``dgl.transform.reverse``."""
        from .transform import reverse
        return reverse(self, share_ndata, share_edata)

    def is_multigraph(self):
        return True

    @property
    def is_readonly(self):
        return self._readonly

    def readonly(self, readonly_state=True):
        """Set the read-only state in place (``graph.py:3819-3860``)."""
        self._readonly = bool(readonly_state)

    @property
    def nodes(self):
        """``G.nodes()`` (all node ids) and ``G.nodes[ids].data`` (view.py:15-81)."""
        return NodeView(self)

    @property
    def edges(self):
        """``G.edges(form, order)`` and ``G.edges[eids or (u, v)].data`` (view.py:83-150)."""
        return EdgeView(self)

    def edge_ids(self, u, v, force_multi=None, return_uv=False):
        """Ids of the edges u[i] -> v[i] (graph.py:399-470); a scalar side broadcasts.
        Every edge of a pair is returned, in id order, pair after pair; with
        ``return_uv`` also their endpoints."""
        us, vs = _to_index_array(u, "u"), _to_index_array(v, "v")
        if us.shape[0] == 1 and vs.shape[0] > 1:
            us = np.full(vs.shape, us[0], np.int64)
        if vs.shape[0] == 1 and us.shape[0] > 1:
            vs = np.full(us.shape, vs[0], np.int64)
        if us.shape != vs.shape:
            raise DGLError("u and v must have the same length")
        src, dst, _ = self._graph.edges()
        n = max(self.number_of_nodes(), 1)
        key = src * n + dst
        order = np.argsort(key, kind="stable")
        q = us * n + vs
        lo = np.searchsorted(key[order], q, "left")
        hi = np.searchsorted(key[order], q, "right")
        if np.any(hi == lo):
            i = int(np.nonzero(hi == lo)[0][0])
            raise DGLError("Edge (%d, %d) does not exist" % (us[i], vs[i]))
        eids = np.concatenate([order[a:b] for a, b in zip(lo, hi)]) if len(q) else \
            np.empty(0, np.int64)
        e = th.from_numpy(eids.astype(np.int64))
        if return_uv:
            return th.from_numpy(src[eids].copy()), th.from_numpy(dst[eids].copy()), e
        return e

    def edge_id(self, u, v, force_multi=None, return_array=False):
        e = self.edge_ids([u], [v])
        return e if return_array or e.shape[0] != 1 else int(e[0])

    # ---- feature access by rows (graph.py:1870-2060) -----------------------------
    def _rows(self, frame, sel, data, num_rows, inplace):
        for k, val in data.items():
            if not isinstance(val, th.Tensor):
                raise DGLError("Feature %s must be a torch tensor" % k)
            if is_all(sel):
                frame[k] = val
                continue
            idx = th.as_tensor(sel, device=val.device)
            if val.shape[0] != idx.shape[0]:
                raise DGLError("Expected %d rows for feature %s, got %d"
                               % (idx.shape[0], k, val.shape[0]))
            if k in frame:
                base = frame[k]
                if inplace:
                    base.index_copy_(0, idx.to(base.device), val.to(base.device, base.dtype))
                    continue
                frame._cols[k] = base.index_copy(0, idx.to(base.device), val.to(base.device, base.dtype))
            else:
                ids = th.arange(num_rows, device=val.device)
                frame._cols[k] = frame.init_rows(k, val, ids).index_copy(0, idx, val)

    def get_n_repr(self, u=ALL):
        if is_all(u):
            return dict(self._node_frame)
        idx = _to_index_array(u, "u")
        return {k: v[th.as_tensor(idx, device=v.device)] for k, v in self._node_frame.items()}

    def set_n_repr(self, data, u=ALL, inplace=False):
        self._rows(self._node_frame, u if is_all(u) else _to_index_array(u, "u"), data,
                   self.number_of_nodes(), inplace)

    def pop_n_repr(self, key):
        return self._node_frame.pop(key)

    def get_e_repr(self, edges=ALL):
        if is_all(edges):
            return dict(self._edge_frame)
        eid = self._resolve_edges(edges)[2]
        return {k: v[th.as_tensor(eid, device=v.device)] for k, v in self._edge_frame.items()}

    def set_e_repr(self, data, edges=ALL, inplace=False):
        sel = edges if is_all(edges) else self._resolve_edges(edges)[2]
        self._rows(self._edge_frame, sel, data, self.number_of_edges(), inplace)

    def pop_e_repr(self, key):
        return self._edge_frame.pop(key)

    def set_n_initializer(self, initializer, field=None):
        """Initializer of node features (graph.py:1700-1730): ``field`` None sets the
        default of every column."""
        self._node_frame.set_initializer(initializer, field)

    def set_e_initializer(self, initializer, field=None):
        self._edge_frame.set_initializer(initializer, field)

    def clear(self):
        """Remove every node, edge, feature and pending message (graph.py:1190)."""
        self._graph = GraphIndex(0)
        self._node_frame = Frame(self.number_of_nodes, None, self._node_frame._inits)
        self._edge_frame = Frame(self.number_of_edges, None, self._edge_frame._inits)
        self._msg_frame, self._msg_ind = {}, None

    def _get_msg_index(self):
        """Pending-message indicator per edge id (graph.py:_get_msg_index), as int64."""
        ind = getattr(self, "_msg_ind", None)
        if ind is None or ind.shape[0] != self.number_of_edges():
            return np.zeros(self.number_of_edges(), np.int64)
        return ind.astype(np.int64)

    def all_edges(self, form="uv", order=None):
        src, dst, eid = self._graph.edges()
        s, d, e = th.from_numpy(src.copy()), th.from_numpy(dst.copy()), th.from_numpy(eid.copy())
        if form == "uv":
            return s, d
        if form == "eid":
            return e
        if form == "all":
            return s, d, e
        raise DGLError("Invalid form: %s" % form)

    def in_degrees(self, v=ALL):
        d = th.from_numpy(self._graph.in_degrees())
        return d if is_all(v) else d[th.as_tensor(_to_index_array(v, "v"))]

    def out_degrees(self, v=ALL):
        d = th.from_numpy(self._graph.out_degrees())
        return d if is_all(v) else d[th.as_tensor(_to_index_array(v, "v"))]

    def _device_degrees(self, device, direction):
        """In- ("in") or out- ("out") degrees of all nodes as a device tensor, from
        the cached device CSRs (no host round trip; used by GraphConv's norm)."""
        gidx = self._graph.get_immutable_gidx(device)
        return (gidx.in_csr if direction == "in" else gidx.out_csr).degrees()

    def in_degree(self, v):
        return int(self.in_degrees([v])[0])

    def out_degree(self, v):
        return int(self.out_degrees([v])[0])

    def _incident(self, nodes, by_dst, form):
        """Edges of each queried node in query order, each node's edges in id order
        (graph_index.py in_edges / out_edges: one CSR row per node)."""
        q = _to_index_array(nodes, "v")
        src, dst, eid = self._graph.edges()
        key = dst if by_dst else src
        order = np.argsort(key, kind="stable")
        lo = np.searchsorted(key[order], q, "left")
        hi = np.searchsorted(key[order], q, "right")
        sel = np.concatenate([order[a:b] for a, b in zip(lo, hi)]) if len(q) else \
            np.empty(0, np.int64)
        s, d, e = (th.from_numpy(a[sel].copy()) for a in (src, dst, eid))
        return {"uv": (s, d), "eid": e, "all": (s, d, e)}[form]

    def in_edges(self, v, form="uv"):
        return self._incident(v, True, form)

    def out_edges(self, u, form="uv"):
        return self._incident(u, False, form)

    def adjacency_matrix_scipy(self, transpose=False, fmt="csr", return_edge_ids=None):
        """(graph.py:3567-3599) A row is a destination and a column a source by
        default (DGL 0.4); ``transpose=True`` puts sources on the rows.  Entries
        count parallel edges (``return_edge_ids`` is accepted and ignored: the
        values are ones)."""
        import scipy.sparse as sp
        src, dst, _ = self._graph.edges()
        n = self.number_of_nodes()
        r, c = (src, dst) if transpose else (dst, src)
        m = sp.coo_matrix((np.ones(len(src), np.float32), (r, c)), shape=(n, n))
        return m.asformat(fmt)

    def adjacency_matrix(self, transpose=False, ctx=None):
        """(graph.py:3601-3640) torch sparse COO adjacency, destination rows by
        default; ``ctx`` a torch device."""
        src, dst, _ = self._graph.edges()
        n = self.number_of_nodes()
        s, d = th.from_numpy(np.asarray(src)), th.from_numpy(np.asarray(dst))
        idx = th.stack([s, d] if transpose else [d, s])
        m = th.sparse_coo_tensor(idx, th.ones(len(src)), (n, n))
        return m if ctx is None else m.to(ctx)

    # ---- features ---------------------------------------------------------------
    @property
    def ndata(self):
        return self._node_frame

    @property
    def edata(self):
        return self._edge_frame

    @property
    def srcdata(self):
        return self._node_frame

    @property
    def dstdata(self):
        return self._node_frame

    def local_var(self):
        """Shallow copy whose feature writes do not leak out (graph.py:local_var)."""
        g = DGLGraph.__new__(DGLGraph)
        g._graph = self._graph
        g._readonly = self._readonly
        g._node_frame = Frame(g.number_of_nodes, self._node_frame._cols, self._node_frame._inits)
        g._edge_frame = Frame(g.number_of_edges, self._edge_frame._cols, self._edge_frame._inits)
        for attr in ("_message_func", "_reduce_func", "_apply_node_func", "_apply_edge_func"):
            if hasattr(self, attr):
                setattr(g, attr, getattr(self, attr))
        return g

    def local_scope(self):
        import contextlib

        @contextlib.contextmanager
        def scope():
            old_n, old_e = self._node_frame, self._edge_frame
            self._node_frame = old_n.clone()
            self._edge_frame = old_e.clone()
            try:
                yield
            finally:
                self._node_frame, self._edge_frame = old_n, old_e
        return scope()

    def to(self, device):
        g = self.local_var()
        for k, v in list(g._node_frame._cols.items()):
            g._node_frame._cols[k] = v.to(device)
        for k, v in list(g._edge_frame._cols.items()):
            g._edge_frame._cols[k] = v.to(device)
        return g

    # ---- message passing ----------------------------------------------------------
    def _device(self, *frames):
        for fr in frames:
            for v in fr.values():
                return v.device
        return th.device("cuda", th.cuda.current_device()) if th.cuda.is_available() else th.device("cpu")

    def _gidx(self, device):
        return self._graph.get_immutable_gidx(device)

    @staticmethod
    def _as_list(f):
        if f is None:
            return []
        return list(f) if isinstance(f, (list, tuple)) else [f]

    def _builtin_reduce(self, gidx, mfuncs, rfuncs, src_frame, edge_frame, out_size,
                        edge_map=None, udf_msgs=None):
        """One kernel per (message, reducer) pair (scheduler.py:905-917).  With a
        user-defined message function the messages were materialised first
        (``udf_msgs``: field -> per-edge tensor indexed by parent edge id) and each
        reducer runs as ``copy_e`` over them (scheduler.py:919-960)."""
        fld2mfunc = {fn.out_field: fn for fn in mfuncs if isinstance(fn, MessageFunction)}
        out = {}
        for rfn in rfuncs:
            if udf_msgs is not None:
                if rfn.msg_field not in udf_msgs:
                    raise DGLError('Reduce function requires message field "%s", but the '
                                   'message function does not generate it.' % rfn.msg_field)
                out[rfn.out_field] = B.copy_reduce(rfn.name, gidx, TargetCode.EDGE,
                                                   udf_msgs[rfn.msg_field], out_size)
                continue
            if rfn.msg_field not in fld2mfunc:
                raise DGLError('Reduce function requires message field "%s", but no message '
                               'function generates it.' % rfn.msg_field)
            mfn = fld2mfunc[rfn.msg_field]
            out[rfn.out_field] = mfn._invoke(gidx, src_frame, src_frame, edge_frame, out_size,
                                             None, None, edge_map, None, reducer=rfn.name)
        return out

    @staticmethod
    def _is_udf(mfuncs):
        return len(mfuncs) == 1 and not isinstance(mfuncs[0], MessageFunction)

    @staticmethod
    def _is_udf_reduce(rfuncs):
        return len(rfuncs) == 1 and not isinstance(rfuncs[0], ReduceFunction)

    def _check_builtin(self, mfuncs, rfuncs):
        if not mfuncs:
            raise DGLError("A message function is required (pass one or call "
                           "register_message_func)")
        self._check_reduce(rfuncs)
        if not self._is_udf(mfuncs):
            for f in mfuncs:
                if not isinstance(f, MessageFunction):
                    raise DGLError("A list of message functions must hold builtins "
                                   "(dgl.function.*) only")

    @staticmethod
    def _check_reduce(rfuncs):
        if not rfuncs:
            raise DGLError("A reduce function is required (pass one or call "
                           "register_reduce_func)")
        if len(rfuncs) > 1 or isinstance(rfuncs[0], ReduceFunction):
            for f in rfuncs:
                if not isinstance(f, ReduceFunction):
                    raise DGLError("A list of reduce functions must hold builtins "
                                   "(dgl.function.*) only")
        elif not callable(rfuncs[0]):
            raise DGLError("Invalid reduce function: %r" % (rfuncs[0],))

    def _messages(self, gidx, mfuncs, s, d, e, dev):
        """Every message of the selected edges as per-edge tensors indexed by (parent)
        edge id: builtins as one reducer-"none" kernel each, a UDF on an EdgeBatch."""
        if self._is_udf(mfuncs):
            return self._udf_messages(mfuncs[0], s, d, e, dev)
        m = self.number_of_edges()
        return {f.out_field: f._invoke(gidx, self._node_frame, self._node_frame,
                                       self._edge_frame, m, reducer="none") for f in mfuncs}

    def _reduce(self, gidx, mfuncs, rfuncs, edges, dev, msgs=None):
        """Reduce messages on every node of ``gidx`` (the whole graph or an in-edge
        subgraph).  Builtin reducers: one kernel per (message, reducer) pair, or copy_e
        over materialised messages.  A reduce UDF: degree bucketing
        (runtime/degree_bucketing.py:12-80).  ``edges`` returns the selected edges as
        device (src, dst, eid) tensors in edge-id order."""
        if self._is_udf_reduce(rfuncs):
            s, d, e = edges()
            if msgs is None:
                msgs = self._messages(gidx, mfuncs, s, d, e, dev)
            return self._degree_bucket_reduce(rfuncs[0], msgs, d, e, dev)
        if msgs is None and self._is_udf(mfuncs):
            s, d, e = edges()
            msgs = self._udf_messages(mfuncs[0], s, d, e, dev)
        return self._builtin_reduce(gidx, mfuncs, rfuncs, self._node_frame, self._edge_frame,
                                    self.number_of_nodes(), udf_msgs=msgs)

    def _degree_bucket_reduce(self, rfunc, msgs, d, e, dev):
        """runtime/degree_bucketing.py + src/scheduler/scheduler.cc:13-100 on the device:
        destination nodes grouped by in-degree, one reduce-UDF call per bucket on a
        (nodes, degree, ...) mailbox whose messages keep their edge-id order, results
        merged by node id.  Rows of nodes that received nothing stay zero (the zero
        initializer of the reference's zero-degree bucket)."""
        n = self.number_of_nodes()
        d = d.long()
        order = th.argsort(d, stable=True)
        ds, es = d[order], e.long()[order]
        deg = th.bincount(ds, minlength=n)
        starts = th.cumsum(deg, 0) - deg
        out = {}
        for dv in th.unique(deg).tolist():
            if dv == 0:
                continue
            nodes = th.nonzero(deg == dv).squeeze(1)
            pos = starts[nodes].unsqueeze(1) + th.arange(dv, device=dev)
            mids = es[pos]
            mail = {k: t[mids] for k, t in msgs.items()}
            nb = NodeBatch(nodes, {k: t[nodes] for k, t in self._node_frame.items()}, mail)
            for k, t in rfunc(nb).items():
                if k not in out:
                    out[k] = t.new_zeros((n,) + tuple(t.shape[1:]))
                out[k] = out[k].index_copy(0, nodes, t)
        zero = th.nonzero(deg == 0).squeeze(1)
        if out and zero.numel():
            # zero-degree rows: the node frame's initializer for the field
            # (degree_bucketing.py:73-79, ir NEW_DICT)
            for k in out:
                out[k] = out[k].index_copy(0, zero, self._node_frame.init_rows(k, out[k], zero))
        return out

    # ---- registered defaults (graph.py:2458-2548) -------------------------------------
    def register_message_func(self, func):
        """Default message function of update_all / send / pull / push / send_and_recv."""
        self._message_func = func

    def register_reduce_func(self, func):
        """Default reduce function of update_all / recv / pull / push / send_and_recv."""
        self._reduce_func = func

    def register_apply_node_func(self, func):
        """Default node update applied after a reduce."""
        self._apply_node_func = func

    def register_apply_edge_func(self, func):
        """Default edge function of apply_edges."""
        self._apply_edge_func = func

    def _default(self, func, attr):
        if isinstance(func, str) and func == "default":
            return getattr(self, attr, None)
        return func

    def _defaults(self, message_func, reduce_func, apply_node_func):
        return (self._default(message_func, "_message_func"),
                self._default(reduce_func, "_reduce_func"),
                self._default(apply_node_func, "_apply_node_func"))

    def _udf_messages(self, func, s, d, e, dev):
        """Materialise a message UDF on the selected edges as full per-edge tensors
        indexed by edge id (rows of unselected edges are zero and never read)."""
        eb = EdgeBatch(s, d, e, {k: v[s] for k, v in self._node_frame.items()},
                       {k: v[d] for k, v in self._node_frame.items()},
                       {k: v[e] for k, v in self._edge_frame.items()})
        m = self.number_of_edges()
        out = {}
        for k, v in func(eb).items():
            if v.shape[0] == m and e.shape[0] == m and bool((e == th.arange(m, device=e.device)).all()):
                out[k] = v
            else:
                out[k] = v.new_zeros((m,) + tuple(v.shape[1:])).index_copy(0, e, v)
        return out

    def update_all(self, message_func="default", reduce_func="default",
                   apply_node_func="default"):
        """Send messages along all edges and reduce them on every node."""
        message_func, reduce_func, apply_node_func = self._defaults(
            message_func, reduce_func, apply_node_func)
        mfuncs, rfuncs = self._as_list(message_func), self._as_list(reduce_func)
        self._check_builtin(mfuncs, rfuncs)
        if self.number_of_nodes() == 0:
            return
        if self.number_of_edges() == 0:  # scheduler.py:214-219: every node has zero
            if apply_node_func is not None:  # in-degree, downgrade to apply_nodes
                self.apply_nodes(apply_node_func)
            return
        dev = self._device(self._node_frame, self._edge_frame)
        gidx = self._gidx(dev)
        res = self._reduce(gidx, mfuncs, rfuncs, lambda: self._edge_tensors(ALL, dev), dev)
        if apply_node_func is not None:
            nb = NodeBatch(self.nodes().to(dev), dict(self._node_frame, **res))
            res.update(apply_node_func(nb))
        for k, v in res.items():
            self._node_frame[k] = v

    def _subgraph_index(self, src, dst, eid):
        """Index over all nodes holding only the given edges; CSR data = parent eids."""
        sub = GraphIndex(self.number_of_nodes())
        sub.add_edges(src, dst)
        sub._parent_eid = eid
        return sub

    def _write_partial(self, res, recv_nodes, apply_node_func, dev, inplace=False):
        """Write reduced rows of ``recv_nodes`` (sorted, unique) into the node frame,
        after the optional apply function (scheduler.py:_apply_with_accum); with
        ``inplace`` into the frame's existing tensors (WRITE_ROW_INPLACE_)."""
        v = th.as_tensor(np.unique(recv_nodes), device=dev)
        if apply_node_func is not None:
            data = {k: t[v] for k, t in self._node_frame.items()}
            data.update({k: t[v] for k, t in res.items()})
            nb = NodeBatch(v, data)
            for k, t in apply_node_func(nb).items():
                res[k] = th.zeros((self.number_of_nodes(),) + tuple(t.shape[1:]), dtype=t.dtype,
                                  device=dev).index_copy(0, v, t)
        self._rows(self._node_frame, v.cpu().numpy(), {k: t[v] for k, t in res.items()},
                   self.number_of_nodes(), inplace)

    def _partial_reduce(self, src, dst, eid, message_func, reduce_func, apply_node_func,
                        recv_nodes, inplace=False):
        message_func, reduce_func, apply_node_func = self._defaults(
            message_func, reduce_func, apply_node_func)
        mfuncs, rfuncs = self._as_list(message_func), self._as_list(reduce_func)
        self._check_builtin(mfuncs, rfuncs)
        dev = self._device(self._node_frame, self._edge_frame)
        sub = _PartialIndex(self.number_of_nodes(), src, dst, eid, bits=self._graph._bits)
        gidx = sub.get_immutable_gidx(dev)
        res = self._reduce(gidx, mfuncs, rfuncs,
                           lambda: (th.as_tensor(src, device=dev), th.as_tensor(dst, device=dev),
                                    th.as_tensor(eid, device=dev)), dev)
        self._write_partial(res, recv_nodes, apply_node_func, dev, inplace)

    def pull(self, v, message_func="default", reduce_func="default", apply_node_func="default",
             inplace=False):
        """Pull messages from the in-edges of ``v`` and reduce them on ``v``."""
        vs = _to_index_array(v, "v")
        src, dst, eid = self._graph.edges()
        mask = np.isin(dst, vs)
        if not mask.any():  # scheduler.py:472-476: downgrade to apply_nodes
            apply_node_func = self._default(apply_node_func, "_apply_node_func")
            if apply_node_func is not None:
                self.apply_nodes(apply_node_func, vs, inplace)
            return
        self._partial_reduce(src[mask], dst[mask], eid[mask], message_func, reduce_func,
                             apply_node_func, vs, inplace)

    def send_and_recv(self, edges, message_func="default", reduce_func="default",
                      apply_node_func="default", inplace=False):
        """Send messages along ``edges`` (eids or (u, v)) and reduce on their destinations."""
        src, dst, eid = self._resolve_edges(edges)
        if len(eid) == 0:
            return
        self._partial_reduce(src, dst, eid, message_func, reduce_func, apply_node_func, dst,
                             inplace)

    def push(self, u, message_func="default", reduce_func="default", apply_node_func="default",
             inplace=False):
        """Send messages along the out-edges of ``u`` and reduce on their destinations
        (graph.py:3124, scheduler.py:417-449)."""
        us = _to_index_array(u, "u")
        src, dst, eid = self._graph.edges()
        mask = np.isin(src, us)
        if not mask.any():
            return
        self._partial_reduce(src[mask], dst[mask], eid[mask], message_func, reduce_func,
                             apply_node_func, dst[mask], inplace)

    # ---- two-phase send / recv (graph.py:2749-2960, scheduler.py:31-129) ---------------
    def send(self, edges=ALL, message_func="default"):
        """Compute messages on ``edges`` and keep them until a ``recv`` consumes them."""
        message_func = self._default(message_func, "_message_func")
        mfuncs = self._as_list(message_func)
        if not mfuncs:
            raise DGLError("A message function is required (pass one or call "
                           "register_message_func)")
        m = self.number_of_edges()
        if m == 0:
            return
        dev = self._device(self._node_frame, self._edge_frame)
        if self._is_udf(mfuncs):
            s_, d_, e = self._edge_tensors(edges, dev)
            msgs = self._udf_messages(mfuncs[0], s_, d_, e, dev)
        else:
            if is_all(edges):
                gidx = self._gidx(dev)
                e = th.arange(m, device=dev)
            else:
                src, dst, eid = self._resolve_edges(edges)
                gidx = _PartialIndex(self.number_of_nodes(), src, dst, eid,
                                     bits=self._graph._bits).get_immutable_gidx(dev)
                e = th.as_tensor(eid, device=dev)
            msgs = self._messages(gidx, mfuncs, None, None, e, dev)
        if not hasattr(self, "_msg_frame") or self._msg_frame is None:
            self._msg_frame = {}
        ind = getattr(self, "_msg_ind", None)
        if ind is None or ind.shape[0] != m:
            ind = np.zeros(m, bool)
        for k, t in msgs.items():
            old = self._msg_frame.get(k)
            if old is None or old.shape != t.shape:
                self._msg_frame[k] = t
            else:
                self._msg_frame[k] = old.index_copy(0, e, t[e])
        ind[e.cpu().numpy()] = True
        self._msg_ind = ind

    def recv(self, v=ALL, reduce_func="default", apply_node_func="default", inplace=False):
        """Reduce the pending messages of the in-edges of ``v`` onto ``v``; messages are
        consumed (scheduler.py:72-129).  Nodes of ``v`` without a pending message get
        the reducer's value for an empty row."""
        reduce_func = self._default(reduce_func, "_reduce_func")
        apply_node_func = self._default(apply_node_func, "_apply_node_func")
        rfuncs = self._as_list(reduce_func)
        self._check_reduce(rfuncs)
        vs = np.arange(self.number_of_nodes()) if is_all(v) else _to_index_array(v, "v")
        ind = getattr(self, "_msg_ind", None)
        src, dst, eid = self._graph.edges()
        mask = np.isin(dst, vs)
        if ind is not None and ind.shape[0] == len(eid):
            mask &= ind[eid]
        else:
            mask[:] = False
        if not mask.any():  # scheduler.py:101-107: downgrade to apply_nodes
            if apply_node_func is not None:
                self.apply_nodes(apply_node_func, vs, inplace)
            return
        dev = self._device(self._node_frame, self._edge_frame)
        gidx = _PartialIndex(self.number_of_nodes(), src[mask], dst[mask],
                             eid[mask], bits=self._graph._bits).get_immutable_gidx(dev)
        res = self._reduce(gidx, [], rfuncs,
                           lambda: (th.as_tensor(src[mask], device=dev),
                                    th.as_tensor(dst[mask], device=dev),
                                    th.as_tensor(eid[mask], device=dev)), dev,
                           msgs=self._msg_frame)
        self._write_partial(res, vs, apply_node_func, dev, inplace)
        ind[eid[mask]] = False
        if not ind.any():
            self._msg_frame = {}

    def _resolve_edges(self, edges):
        src, dst, eid = self._graph.edges()
        if is_all(edges):
            return src, dst, eid
        nested = getattr(edges, "ndim", 1) > 1 or (
            isinstance(edges, list) and any(isinstance(x, (list, tuple, np.ndarray, th.Tensor))
                                            for x in edges))
        if nested:  # graph.py:2780 (utils.toindex rejects 2-D input)
            raise DGLError("Edges must be edge ids or a (u, v) tuple, got a nested sequence")
        if isinstance(edges, tuple) and len(edges) == 2:
            # every edge of each (u, v) pair, a length-1 side broadcast (utils.py:toindex)
            sel = self.edge_ids(edges[0], edges[1]).numpy()
        else:
            sel = _to_index_array(edges, "eid")
        return src[sel], dst[sel], eid[sel]

    def _edge_tensors(self, edges, dev):
        """(src, dst, eid) device tensors of the selected edges."""
        if is_all(edges) and self._graph._device_only is not None:
            s, d = self._graph._device_only
            s, d = s.to(dev).long(), d.to(dev).long()
            return s, d, th.arange(s.shape[0], device=dev)
        src, dst, eid = self._resolve_edges(edges)
        return (th.as_tensor(src, device=dev), th.as_tensor(dst, device=dev),
                th.as_tensor(eid, device=dev))

    def apply_edges(self, func="default", edges=ALL, inplace=False):
        """Compute per-edge features with a builtin (reducer 'none') or a UDF."""
        func = self._default(func, "_apply_edge_func")
        if func is None:
            raise DGLError("An edge function is required (pass one or call "
                           "register_apply_edge_func)")
        dev = self._device(self._node_frame, self._edge_frame)
        if isinstance(func, MessageFunction):
            m = self.number_of_edges()
            if is_all(edges):
                gidx = self._gidx(dev)
                res = func._invoke(gidx, self._node_frame, self._node_frame, self._edge_frame, m,
                                   reducer="none")
            else:
                src, dst, eid = self._resolve_edges(edges)
                sub = _PartialIndex(self.number_of_nodes(), src, dst, eid, bits=self._graph._bits)
                gidx = sub.get_immutable_gidx(dev)
                res = func._invoke(gidx, self._node_frame, self._node_frame, self._edge_frame, m,
                                   reducer="none")
                sel = th.as_tensor(eid, device=dev)
                self._rows(self._edge_frame, np.asarray(eid), {func.out_field: res[sel]}, m,
                           inplace)
                return
            self._edge_frame[func.out_field] = res  # all edges: a new column, never in place
            return
        s, d, e = self._edge_tensors(edges, dev)
        eb = EdgeBatch(s, d, e, {k: v[s] for k, v in self._node_frame.items()},
                       {k: v[d] for k, v in self._node_frame.items()},
                       {k: v[e] for k, v in self._edge_frame.items()})
        out = func(eb)
        if is_all(edges):  # scheduler.py:334-375: all edges are written as new columns
            for k, v in out.items():
                self._edge_frame[k] = v
            return
        self._rows(self._edge_frame, e.cpu().numpy(), out, self.number_of_edges(), inplace)

    def group_apply_edges(self, group_by, func, edges=ALL, inplace=False):
        """Edges grouped by their source (``group_by='src'``) or destination node,
        one UDF call per degree bucket on (nodes, degree, ...) shaped data, edges of
        a node in edge-id order (graph.py:2667-2760, scheduler.py:377-415)."""
        if group_by not in ("src", "dst"):
            raise DGLError("Group_by should be either src or dst")
        dev = self._device(self._node_frame, self._edge_frame)
        s, d, e = self._edge_tensors(edges, dev)
        key = (s if group_by == "src" else d).long()
        order = th.argsort(key, stable=True)
        n = self.number_of_nodes()
        deg = th.bincount(key, minlength=n)
        starts = th.cumsum(deg, 0) - deg
        out = {}
        for dv in th.unique(deg).tolist():
            if dv == 0:
                continue
            nodes = th.nonzero(deg == dv).squeeze(1)
            pos = order[starts[nodes].unsqueeze(1) + th.arange(dv, device=dev)]   # (b, dv)
            bs, bd, be = s[pos], d[pos], e[pos]
            eb = EdgeBatch(bs, bd, be, {k: t[bs] for k, t in self._node_frame.items()},
                           {k: t[bd] for k, t in self._node_frame.items()},
                           {k: t[be] for k, t in self._edge_frame.items()})
            for k, t in func(eb).items():
                if k not in out:
                    out[k] = t.new_zeros((self.number_of_edges(),) + tuple(t.shape[2:]))
                out[k] = out[k].index_copy(0, be.reshape(-1), t.reshape((-1,) + tuple(t.shape[2:])))
        sel = e.cpu().numpy()
        if is_all(edges) and not inplace:
            for k, t in out.items():
                self._edge_frame[k] = t
            return
        self._rows(self._edge_frame, sel, {k: t[e] for k, t in out.items()},
                   self.number_of_edges(), inplace)

    def apply_nodes(self, func="default", v=ALL, inplace=False):
        func = self._default(func, "_apply_node_func")
        if func is None:
            raise DGLError("A node function is required (pass one or call "
                           "register_apply_node_func)")
        dev = self._device(self._node_frame)
        nodes = self.nodes().to(dev) if is_all(v) else th.as_tensor(_to_index_array(v, "v"), device=dev)
        nb = NodeBatch(nodes, {k: t[nodes] for k, t in self._node_frame.items()})
        out = func(nb)
        if is_all(v):  # all nodes: new columns, never in place (test_inplace_update.py:267)
            for k, t in out.items():
                self._node_frame[k] = t
            return
        self._rows(self._node_frame, nodes.cpu().numpy(), out, self.number_of_nodes(), inplace)


class _PartialIndex(GraphIndex):
    """In-edge subgraph over all nodes whose CSR ``data`` holds the parent edge ids,
    so edge features of the parent graph are addressed directly (the reference uses
    relabel maps for the same purpose, spmv.py:146-180)."""
    _eid_is_perm = False

    def __init__(self, n, src, dst, parent_eid, bits=None):
        super().__init__(n)
        self.add_edges(src, dst)
        self._parent = np.asarray(parent_eid, np.int64)
        self._bits = bits  # the parent's forced width (GraphIndex.asbits)

    def bits_needed(self):
        # the CSR data holds parent edge ids: 64-bit once they reach 2^31
        if self._parent.size and int(self._parent.max()) >= 0x7FFFFFFF:
            return 64
        return super().bits_needed()

    def host_csr(self):
        if self._host_csr is None:
            (op, oi, od), (ip, ii, idd) = super().host_csr()
            self._host_csr = ((op, oi, self._parent[od]), (ip, ii, self._parent[idd]))
        return self._host_csr
