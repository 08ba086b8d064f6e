"""Heterographs for the R-GCN path (``python/dgl/heterograph.py``).

The subset a heterogeneous GNN needs on the message-passing path:

* construction -- ``dgl.heterograph({(srctype, etype, dsttype): (u, v)})``,
  ``dgl.graph``, ``dgl.bipartite``, ``dgl.hetero_from_relations``;
* typed storage -- ``g.nodes[ntype].data``, ``g.edges[etype].data``, ``ndata`` /
  ``edata`` for single-type graphs, counts, degrees, ``to_canonical_etype``;
* relation views ``g[etype]`` / ``g[stype, etype, dtype]`` that behave like a
  (bipartite) DGLGraph -- ``srcdata`` / ``dstdata`` / ``edata``, ``update_all``,
  ``send_and_recv``, ``pull``, ``push``, ``send`` / ``recv``, ``apply_nodes``,
  ``apply_edges``, ``local_var``, with builtin or user-defined message / reduce
  functions (UDF reducers by degree bucketing) -- so GraphConv / GATConv /
  edge_softmax run on one relation and ``nn.pytorch.HeteroGraphConv`` composes
  them (``nn/pytorch/hetero.py:112-170``);
* ``update_all(..., etype=)`` and ``multi_update_all(etype_dict, cross_reducer)``
  (``heterograph.py:3570-3656``).

Each relation is a (num_src x num_dst) block on the device (in-CSR + out-CSR
built by the radix-sort ingestion, cached per device), so every message
function of a relation is the same load-balanced HIP kernel as for a
homogeneous graph.  ``multi_update_all`` with the cross-type reducer ``sum``
over ``copy_u`` + ``sum`` messages -- R-GCN's aggregation -- is FUSED: the
relations into one destination type are merged into one block whose columns
index the concatenated source tables, and ONE SpMM computes
sum_r sum_{u->v in r} X_r[u] (the reference loops over the relations and then
merges the per-type frames, ``heterograph.py:3629-3650``, and says so in a
TODO).  Other reducers run one kernel per relation and merge with torch
(sum / max / min / mean / stack, ``merge_frames`` semantics).
"""
from __future__ import annotations

import contextlib
import types
from collections import OrderedDict

import numpy as np
import torch as th

from ._ffi import DGLError
from .function.message import CopyMessageFunction, MessageFunction
from .function.reducer import ReduceFunction, SimpleReduceFunction
from .function.base import TargetCode
from .graph import ALL, EdgeBatch, NodeBatch, is_all
from .graph_index import device_block_gidx

__all__ = ["DGLHeteroGraph", "heterograph", "graph", "bipartite", "hetero_from_relations"]


def _ids(x):
    if isinstance(x, th.Tensor):
        return x.detach().cpu().numpy().astype(np.int64)
    return np.asarray(x, dtype=np.int64).reshape(-1)


def _uv(data):
    """(u, v) from a pair of id sequences or a list of (u, v) pairs."""
    if isinstance(data, tuple) and len(data) == 2:
        return _ids(data[0]), _ids(data[1])
    arr = np.asarray(list(data), dtype=np.int64).reshape(-1, 2)
    return arr[:, 0].copy(), arr[:, 1].copy()


class _Rel:
    """Edges of one canonical edge type and their per-device block index."""

    def __init__(self, src, dst, n_src, n_dst):
        self.src, self.dst = src, dst
        self.n_src, self.n_dst = n_src, n_dst
        self._cache = {}

    def number_of_edges(self):
        return int(self.src.shape[0])

    def edges(self):
        return self.src, self.dst, np.arange(self.src.shape[0], dtype=np.int64)

    def get_immutable_gidx(self, device):
        device = th.device(device)
        if device.type != "cuda":
            raise DGLError("the MI355X engine runs on ROCm devices only; got device %s" % device)
        if device.index is None:
            device = th.device("cuda", th.cuda.current_device())
        key = str(device)
        if key not in self._cache:
            if max(self.n_src, self.n_dst, self.number_of_edges()) >= 0x7FFFFFFF:
                raise DGLError("Unsupported idx bits: 64 (graphs need < 2^31 nodes and edges)")
            s = th.from_numpy(self.src.astype(np.int32)).to(device)
            d = th.from_numpy(self.dst.astype(np.int32)).to(device)
            self._cache[key] = device_block_gidx(self.n_src, self.n_dst, s, d)
        return self._cache[key]


class _NodeSpace:
    def __init__(self, g):
        self._g = g

    def __getitem__(self, ntype):
        return types.SimpleNamespace(data=self._g._nframes[self._g._check_ntype(ntype)])

    def __call__(self, ntype=None):
        return th.arange(self._g.number_of_nodes(ntype), dtype=th.int64)


class _EdgeSpace:
    def __init__(self, g):
        self._g = g

    def __getitem__(self, etype):
        return types.SimpleNamespace(data=self._g._eframes[self._g.to_canonical_etype(etype)])

    def __call__(self, form="uv", etype=None):
        src, dst, eid = self._g._rels[self._g.to_canonical_etype(etype)].edges()
        s, d, e = th.from_numpy(src.copy()), th.from_numpy(dst.copy()), th.from_numpy(eid)
        return {"uv": (s, d), "eid": e, "all": (s, d, e)}[form]


def _merge(tensors, reducer):
    """merge_frames (heterograph.py) for one field."""
    if len(tensors) == 1 and reducer != "stack":
        return tensors[0]
    if reducer == "sum":
        out = tensors[0]
        for t in tensors[1:]:
            out = out + t
        return out
    if reducer == "max":
        return th.stack(tensors, 0).max(0)[0]
    if reducer == "min":
        return th.stack(tensors, 0).min(0)[0]
    if reducer == "mean":
        return th.stack(tensors, 0).mean(0)
    if reducer == "stack":
        return th.stack(tensors, 1)
    raise DGLError("Invalid cross type reducer %s: must be sum, max, min, mean or stack" % reducer)


def _as_list(f):
    return list(f) if isinstance(f, (list, tuple)) else [f]


def _reduce(rel, gidx, mfuncs, rfuncs, srcf, dstf, edgef):
    fld2m = {f.out_field: f for f in mfuncs}
    out = {}
    for r in rfuncs:
        if r.msg_field not in fld2m:
            raise DGLError('Reduce function requires message field "%s", but no message '
                           'function generates it.' % r.msg_field)
        out[r.out_field] = fld2m[r.msg_field]._invoke(gidx, srcf, dstf, edgef, rel.n_dst,
                                                      reducer=r.name)
    return out


def _device_of(*frames):
    for f in frames:
        for v in f.values():
            if isinstance(v, th.Tensor):
                return v.device
    return th.device("cuda", th.cuda.current_device())


def _is_udf(funcs):
    return len(funcs) == 1 and not isinstance(funcs[0], (MessageFunction, ReduceFunction))


def _check_funcs(mfuncs, rfuncs):
    """Builtins (one kernel per message / reduce pair) or ONE user-defined message
    and / or reduce function (heterograph.py:3400-3470 accepts both)."""
    if not _is_udf(mfuncs):
        for f in mfuncs:
            if not isinstance(f, MessageFunction):
                raise DGLError("a list of message functions must hold builtins only")
    if not _is_udf(rfuncs):
        for f in rfuncs:
            if not isinstance(f, ReduceFunction):
                raise DGLError("a list of reduce functions must hold builtins only")


def _rel_edge_ids(rel, u, v):
    """Every edge u[i] -> v[i] of one relation, in id order per pair; a length-1
    side broadcasts (heterograph.py:edge_ids)."""
    us, vs = _ids(u), _ids(v)
    if us.shape[0] == 1 and vs.shape[0] > 1:
        us = np.full(vs.shape, us[0], np.int64)
    if vs.shape[0] == 1 and us.shape[0] > 1:
        vs = np.full(us.shape, vs[0], np.int64)
    if us.shape != vs.shape:
        raise DGLError("u and v must have the same length")
    key = rel.src * max(rel.n_dst, 1) + rel.dst
    order = np.argsort(key, kind="stable")
    q = us * max(rel.n_dst, 1) + vs
    lo, hi = np.searchsorted(key[order], q, "left"), np.searchsorted(key[order], q, "right")
    if np.any(hi == lo):
        i = int(np.nonzero(hi == lo)[0][0])
        raise DGLError("Edge (%d, %d) does not exist" % (us[i], vs[i]))
    return np.concatenate([order[a:b] for a, b in zip(lo, hi)]) if len(q) else \
        np.empty(0, np.int64)


def _select(rel, edges):
    """Edge ids of ``edges``: ALL, ids, or a (u, v) pair of id sequences."""
    if is_all(edges):
        return None
    if isinstance(edges, tuple) and len(edges) == 2:
        return _rel_edge_ids(rel, edges[0], edges[1])
    return _ids(edges)


def _rel_messages(mfuncs, gidx, s, d, srcf, dstf, edgef, m):
    """Messages of the walked edges, one row per edge in the block's edge order."""
    if _is_udf(mfuncs):
        eb = EdgeBatch(s, d, th.arange(m, device=s.device), {k: v[s] for k, v in srcf.items()},
                       {k: v[d] for k, v in dstf.items()}, dict(edgef))
        return dict(mfuncs[0](eb))
    return {f.out_field: f._invoke(gidx, srcf, dstf, edgef, m, reducer="none") for f in mfuncs}


def _bucket_reduce(rfunc, msgs, d, n_dst, dstf):
    """Degree bucketing (runtime/degree_bucketing.py) on the destination side of one
    relation: one UDF call per in-degree on a (nodes, degree, ...) mailbox in edge
    order; rows of nodes without messages are zero."""
    d = d.long()
    order = th.argsort(d, stable=True)
    deg = th.bincount(d, minlength=n_dst)
    starts = th.cumsum(deg, 0) - deg
    out = {}
    for dv in th.unique(deg).tolist():
        if dv == 0:
            continue
        nodes = th.nonzero(deg == dv).squeeze(1)
        mids = order[starts[nodes].unsqueeze(1) + th.arange(dv, device=d.device)]
        nb = NodeBatch(nodes, {k: t[nodes] for k, t in dstf.items()},
                       {k: t[mids] for k, t in msgs.items()})
        for k, t in rfunc(nb).items():
            if k not in out:
                out[k] = t.new_zeros((n_dst,) + tuple(t.shape[1:]))
            out[k] = out[k].index_copy(0, nodes, t)
    return out


def _rel_reduce(rel, mfuncs, rfuncs, srcf, dstf, edgef, sel=None, msgs=None):
    """Reduce the messages of one relation's edges (all, or the ids ``sel``) onto
    its destination nodes: builtin pairs as one HIP kernel each, a UDF message as
    materialised rows reduced by ``copy_e`` kernels, a UDF reducer by degree
    bucketing.  ``msgs`` (rows in ``sel`` order) replaces the message function."""
    from . import backend as B
    dev = _device_of(srcf, dstf, edgef)
    if sel is None:
        gidx = rel.get_immutable_gidx(dev)
        s = th.from_numpy(rel.src).to(dev)
        d = th.from_numpy(rel.dst).to(dev)
        ef = edgef
    else:
        s = th.from_numpy(rel.src[sel]).to(dev)
        d = th.from_numpy(rel.dst[sel]).to(dev)
        gidx = device_block_gidx(rel.n_src, rel.n_dst, s.int(), d.int())
        st = th.from_numpy(sel).to(dev)
        ef = {k: v[st] for k, v in edgef.items()}
    m = int(s.shape[0])
    if _is_udf(rfuncs):
        if msgs is None:
            msgs = _rel_messages(mfuncs, gidx, s, d, srcf, dstf, ef, m)
        return _bucket_reduce(rfuncs[0], msgs, d, rel.n_dst, dstf)
    if msgs is None and _is_udf(mfuncs):
        msgs = _rel_messages(mfuncs, gidx, s, d, srcf, dstf, ef, m)
    if msgs is not None:
        out = {}
        for r in rfuncs:
            if r.msg_field not in msgs:
                raise DGLError('Reduce function requires message field "%s", but the '
                               'message function does not generate it.' % r.msg_field)
            out[r.out_field] = B.copy_reduce(r.name, gidx, TargetCode.EDGE,
                                             msgs[r.msg_field].contiguous(), rel.n_dst)
        return out
    return _reduce(rel, gidx, mfuncs, rfuncs, srcf, dstf, ef)


def _write_rows(frame, v, res, n):
    """Rows ``v`` (device ids) of ``res`` into a node frame (a dict of columns)."""
    for k, t in res.items():
        base = frame[k] if k in frame else t.new_zeros((n,) + tuple(t.shape[1:]))
        frame[k] = base.index_copy(0, v, t[v].to(base.dtype))


class DGLHeteroGraph:
    """A graph with node types and edge types (``heterograph.py:DGLHeteroGraph``)."""

    def __init__(self, rels, num_nodes):
        self._ntypes = list(num_nodes.keys())
        self._num_nodes = dict(num_nodes)
        self._cetypes = list(rels.keys())
        self._rels = OrderedDict()
        for (s, e, d), (u, v) in rels.items():
            u, v = _ids(u), _ids(v)
            if u.shape != v.shape:
                raise DGLError("edge type %s: src and dst id arrays differ in length" % e)
            if u.size and (u.min() < 0 or u.max() >= num_nodes[s] or v.min() < 0 or
                           v.max() >= num_nodes[d]):
                raise DGLError("edge type %s: node id out of range" % e)
            self._rels[(s, e, d)] = _Rel(u, v, num_nodes[s], num_nodes[d])
        self._nframes = {t: {} for t in self._ntypes}
        self._eframes = {c: {} for c in self._cetypes}
        self._fused = {}

    # ---- metadata ---------------------------------------------------------------
    @property
    def ntypes(self):
        return list(self._ntypes)

    @property
    def etypes(self):
        return [e for _, e, _ in self._cetypes]

    @property
    def canonical_etypes(self):
        return list(self._cetypes)

    @property
    def srctypes(self):
        return list(self._ntypes)

    @property
    def dsttypes(self):
        return list(self._ntypes)

    def _check_ntype(self, ntype):
        if ntype is None:
            if len(self._ntypes) != 1:
                raise DGLError("Node type name must be specified if there are more than one "
                               "node types.")
            return self._ntypes[0]
        if ntype not in self._num_nodes:
            raise DGLError("Node type %s does not exist." % ntype)
        return ntype

    def to_canonical_etype(self, etype):
        if etype is None:
            if len(self._cetypes) != 1:
                raise DGLError("Edge type name must be specified if there are more than one "
                               "edge types.")
            return self._cetypes[0]
        if isinstance(etype, tuple):
            if etype not in self._rels:
                raise DGLError("Edge type %s does not exist." % (etype,))
            return etype
        hits = [c for c in self._cetypes if c[1] == etype]
        if len(hits) != 1:
            raise DGLError("Edge type %s is %s." % (etype, "ambiguous" if hits else "not found"))
        return hits[0]

    def get_etype_id(self, etype):
        return self._cetypes.index(self.to_canonical_etype(etype))

    def number_of_nodes(self, ntype=None):
        return self._num_nodes[self._check_ntype(ntype)]

    def number_of_edges(self, etype=None):
        if etype is None and len(self._cetypes) > 1:
            return sum(r.number_of_edges() for r in self._rels.values())
        return self._rels[self.to_canonical_etype(etype)].number_of_edges()

    @property
    def nodes(self):
        return _NodeSpace(self)

    @property
    def edges(self):
        return _EdgeSpace(self)

    @property
    def ndata(self):
        return self._nframes[self._check_ntype(None)]

    @property
    def edata(self):
        return self._eframes[self.to_canonical_etype(None)]

    def in_degrees(self, v=ALL, etype=None):
        r = self._rels[self.to_canonical_etype(etype)]
        d = th.from_numpy(np.bincount(r.dst, minlength=r.n_dst))
        return d if is_all(v) else d[th.as_tensor(_ids(v))]

    def out_degrees(self, v=ALL, etype=None):
        r = self._rels[self.to_canonical_etype(etype)]
        d = th.from_numpy(np.bincount(r.src, minlength=r.n_src))
        return d if is_all(v) else d[th.as_tensor(_ids(v))]

    def __getitem__(self, key):
        return _RelationGraph(self, self.to_canonical_etype(key))

    # ---- single-relation graphs (dgl.graph / dgl.bipartite) used like a DGLGraph by
    # the nn modules: everything goes to the one relation's view
    @property
    def _graph(self):
        return self._rels[self.to_canonical_etype(None)]

    @property
    def srcdata(self):
        return self[None].srcdata

    @property
    def dstdata(self):
        return self[None].dstdata

    def number_of_src_nodes(self):
        return self._graph.n_src

    def number_of_dst_nodes(self):
        return self._graph.n_dst

    def _device_degrees(self, device, direction):
        return self[None]._device_degrees(device, direction)

    def is_homograph(self):
        return len(self._ntypes) == 1 and len(self._cetypes) == 1

    def adjacency_matrix(self, transpose=False, ctx=None, etype=None):
        """(heterograph.py:2134-2180) torch sparse COO adjacency of one relation:
        (num_dst, num_src) with destination rows by default."""
        r = self._rels[self.to_canonical_etype(etype)]
        s, d = th.from_numpy(r.src), th.from_numpy(r.dst)
        idx = th.stack([s, d] if transpose else [d, s])
        shape = (r.n_src, r.n_dst) if transpose else (r.n_dst, r.n_src)
        m = th.sparse_coo_tensor(idx, th.ones(len(r.src)), shape)
        return m if ctx is None else m.to(ctx)

    def local_var(self):
        g = DGLHeteroGraph.__new__(DGLHeteroGraph)
        g.__dict__.update(self.__dict__)
        g._nframes = {t: dict(f) for t, f in self._nframes.items()}
        g._eframes = {c: dict(f) for c, f in self._eframes.items()}
        return g

    @contextlib.contextmanager
    def local_scope(self):
        old_n, old_e = self._nframes, self._eframes
        self._nframes = {t: dict(f) for t, f in old_n.items()}
        self._eframes = {c: dict(f) for c, f in old_e.items()}
        try:
            yield
        finally:
            self._nframes, self._eframes = old_n, old_e

    # ---- message passing --------------------------------------------------------
    def apply_edges(self, func, edges=ALL, etype=None):
        self[self.to_canonical_etype(etype)].apply_edges(func, edges)

    def update_all(self, message_func, reduce_func, apply_node_func=None, etype=None):
        """One relation (``heterograph.py`` update_all with etype)."""
        self[self.to_canonical_etype(etype)].update_all(message_func, reduce_func, apply_node_func)

    def multi_update_all(self, etype_dict, cross_reducer, apply_node_func=None):
        """``heterograph.py:3570-3656``: per-type (msg, reduce[, apply]) then a
        cross-type merge per destination type; the sum of copy_u/sum messages is
        one fused SpMM over the merged relations."""
        groups = OrderedDict()
        for etype, args in etype_dict.items():
            c = self.to_canonical_etype(etype)
            args = tuple(args) + (None,) * (3 - len(args))
            groups.setdefault(c[2], []).append((c,) + args)
        for dtype, items in groups.items():
            res = None
            if cross_reducer == "sum":
                res = self._fused_copy_sum(dtype, items)
            if res is None:
                per_field = OrderedDict()
                for c, mfunc, rfunc, afunc in sorted(items, key=lambda it: self._cetypes.index(it[0])):
                    mfs, rfs = _as_list(mfunc), _as_list(rfunc)
                    _check_funcs(mfs, rfs)
                    rel = self._rels[c]
                    srcf, dstf, edgef = self._nframes[c[0]], self._nframes[c[2]], self._eframes[c]
                    out = _rel_reduce(rel, mfs, rfs, srcf, dstf, edgef)
                    if afunc is not None:
                        nb = NodeBatch(th.arange(rel.n_dst), dict(dstf, **out))
                        out.update(afunc(nb))
                    for k, v in out.items():
                        per_field.setdefault(k, []).append(v)
                res = {k: _merge(v, cross_reducer) for k, v in per_field.items()}
            self._nframes[dtype].update(res)
            if apply_node_func is not None:
                nb = NodeBatch(th.arange(self._num_nodes[dtype]), dict(self._nframes[dtype]))
                self._nframes[dtype].update(apply_node_func(nb))

    def _fused_copy_sum(self, dtype, items):
        """All relations into `dtype` send copy_u(field) and sum into the same
        output field, no per-type apply: one SpMM over the merged block."""
        out_field, srcs = None, []
        for c, mfunc, rfunc, afunc in items:
            if afunc is not None or isinstance(mfunc, (list, tuple)) or isinstance(rfunc, (list, tuple)):
                return None
            if not (isinstance(mfunc, CopyMessageFunction) and mfunc.target == TargetCode.SRC and
                    isinstance(rfunc, SimpleReduceFunction) and rfunc.name == "sum" and
                    rfunc.msg_field == mfunc.out_field):
                return None
            if out_field not in (None, rfunc.out_field):
                return None
            out_field = rfunc.out_field
            if mfunc.in_field not in self._nframes[c[0]]:
                return None
            srcs.append((c, c[0], mfunc.in_field))
        if len(srcs) < 2:
            return None
        tables = list(OrderedDict(((s, f), None) for _, s, f in srcs).keys())
        xs = [self._nframes[s][f] for s, f in tables]
        if any(x.shape[1:] != xs[0].shape[1:] or x.dtype != xs[0].dtype for x in xs):
            return None
        dev = xs[0].device
        key = (dtype, tuple(c for c, _, _ in srcs), tuple(tables), str(dev))
        if key not in self._fused:
            offs, o = {}, 0
            for s, f in tables:
                offs[(s, f)] = o
                o += self._num_nodes[s]
            us = [self._rels[c].src + offs[(s, f)] for c, s, f in srcs]
            vs = [self._rels[c].dst for c, _, _ in srcs]
            u = th.from_numpy(np.concatenate(us).astype(np.int32)).to(dev)
            v = th.from_numpy(np.concatenate(vs).astype(np.int32)).to(dev)
            self._fused[key] = device_block_gidx(o, self._num_nodes[dtype], u, v)
        x = xs[0] if len(xs) == 1 else th.cat(xs, 0)
        from . import backend as B
        return {out_field: B.copy_reduce("sum", self._fused[key], TargetCode.SRC, x,
                                         self._num_nodes[dtype])}


class _RelationGraph:
    """One relation of a heterograph, used like a (bipartite) DGLGraph."""

    def __init__(self, parent, cetype, srcf=None, dstf=None, edgef=None):
        self._parent = parent
        self._cetype = cetype
        self._graph = parent._rels[cetype]
        s, _, d = cetype
        self.srcdata = parent._nframes[s] if srcf is None else srcf
        self.dstdata = parent._nframes[d] if dstf is None else dstf
        self.edata = parent._eframes[cetype] if edgef is None else edgef

    @property
    def canonical_etypes(self):
        return [self._cetype]

    @property
    def ndata(self):
        if self._cetype[0] != self._cetype[2]:
            raise DGLError("ndata is ambiguous on a bipartite relation; use srcdata / dstdata")
        return self.srcdata

    def number_of_src_nodes(self):
        return self._graph.n_src

    def number_of_dst_nodes(self):
        return self._graph.n_dst

    def number_of_nodes(self):
        """Destination count (the node set messages are reduced on)."""
        return self._graph.n_dst

    def number_of_edges(self):
        return self._graph.number_of_edges()

    def edges(self, form="uv", order=None):
        return _EdgeSpace(self._parent)(form, self._cetype)

    def in_degrees(self, v=ALL):
        return self._parent.in_degrees(v, self._cetype)

    def out_degrees(self, v=ALL):
        return self._parent.out_degrees(v, self._cetype)

    def _device_degrees(self, device, direction):
        gidx = self._graph.get_immutable_gidx(device)
        return (gidx.in_csr if direction == "in" else gidx.out_csr).degrees()

    def local_var(self):
        same = self._cetype[0] == self._cetype[2]
        src = dict(self.srcdata)
        return _RelationGraph(self._parent, self._cetype, src, src if same else dict(self.dstdata),
                              dict(self.edata))

    @contextlib.contextmanager
    def local_scope(self):
        old = (self.srcdata, self.dstdata, self.edata)
        same = self._cetype[0] == self._cetype[2]
        self.srcdata = dict(old[0])
        self.dstdata = self.srcdata if same else dict(old[1])
        self.edata = dict(old[2])
        try:
            yield
        finally:
            self.srcdata, self.dstdata, self.edata = old

    def update_all(self, message_func, reduce_func, apply_node_func=None):
        mfs, rfs = _as_list(message_func), _as_list(reduce_func)
        _check_funcs(mfs, rfs)
        rel = self._graph
        if rel.number_of_edges() == 0:  # scheduler.py:216-222: downgrade to apply
            if apply_node_func is not None:
                self.apply_nodes(apply_node_func)
            return
        out = _rel_reduce(rel, mfs, rfs, self.srcdata, self.dstdata, self.edata)
        if apply_node_func is not None:
            nb = NodeBatch(th.arange(rel.n_dst), dict(self.dstdata, **out))
            out.update(apply_node_func(nb))
        self.dstdata.update(out)

    def apply_nodes(self, func, v=ALL):
        """On the destination nodes of the relation."""
        dev = _device_of(self.dstdata)
        nodes = th.arange(self._graph.n_dst, device=dev) if is_all(v) else \
            th.as_tensor(_ids(v), device=dev)
        out = func(NodeBatch(nodes, {k: t[nodes] for k, t in self.dstdata.items()}))
        if is_all(v):
            self.dstdata.update(out)
        else:
            _write_rows(self.dstdata, nodes, {k: t.new_zeros((self._graph.n_dst,) +
                                                             tuple(t.shape[1:])).index_copy(0, nodes, t)
                                              for k, t in out.items()}, self._graph.n_dst)

    def _partial(self, sel, recv, mfs, rfs, afunc, msgs=None):
        """Reduce the edges ``sel`` onto the destination nodes ``recv`` (sorted,
        unique numpy ids), apply, write their rows (scheduler.py:_apply_with_accum)."""
        rel = self._graph
        dev = _device_of(self.srcdata, self.dstdata, self.edata)
        out = _rel_reduce(rel, mfs, rfs, self.srcdata, self.dstdata, self.edata, sel, msgs)
        v = th.as_tensor(recv, device=dev)
        if afunc is not None:
            data = {k: t[v] for k, t in self.dstdata.items()}
            data.update({k: t[v] for k, t in out.items()})
            for k, t in afunc(NodeBatch(v, data)).items():
                out[k] = t.new_zeros((rel.n_dst,) + tuple(t.shape[1:])).index_copy(0, v, t)
        _write_rows(self.dstdata, v, out, rel.n_dst)

    def send_and_recv(self, edges, message_func, reduce_func, apply_node_func=None):
        mfs, rfs = _as_list(message_func), _as_list(reduce_func)
        _check_funcs(mfs, rfs)
        sel = _select(self._graph, edges)
        sel = np.arange(self._graph.number_of_edges()) if sel is None else sel
        if sel.size == 0:
            return
        self._partial(sel, np.unique(self._graph.dst[sel]), mfs, rfs, apply_node_func)

    def pull(self, v, message_func, reduce_func, apply_node_func=None):
        mfs, rfs = _as_list(message_func), _as_list(reduce_func)
        _check_funcs(mfs, rfs)
        vs = np.unique(_ids(v))
        sel = np.nonzero(np.isin(self._graph.dst, vs))[0]
        if sel.size == 0:  # scheduler.py:472-476
            if apply_node_func is not None:
                self.apply_nodes(apply_node_func, vs)
            return
        self._partial(sel, vs, mfs, rfs, apply_node_func)

    def push(self, u, message_func, reduce_func, apply_node_func=None):
        mfs, rfs = _as_list(message_func), _as_list(reduce_func)
        _check_funcs(mfs, rfs)
        sel = np.nonzero(np.isin(self._graph.src, _ids(u)))[0]
        if sel.size == 0:
            return
        self._partial(sel, np.unique(self._graph.dst[sel]), mfs, rfs, apply_node_func)

    def send(self, edges=ALL, message_func=None):
        """Messages of ``edges`` kept on the relation until ``recv`` consumes them."""
        rel = self._graph
        mfs = _as_list(message_func)
        _check_funcs(mfs, [])
        sel = _select(rel, edges)
        sel = np.arange(rel.number_of_edges()) if sel is None else sel
        if sel.size == 0:
            return
        dev = _device_of(self.srcdata, self.dstdata, self.edata)
        s = th.from_numpy(rel.src[sel]).to(dev)
        d = th.from_numpy(rel.dst[sel]).to(dev)
        gidx = device_block_gidx(rel.n_src, rel.n_dst, s.int(), d.int())
        st = th.from_numpy(sel).to(dev)
        msgs = _rel_messages(mfs, gidx, s, d, self.srcdata, self.dstdata,
                             {k: t[st] for k, t in self.edata.items()}, int(sel.size))
        m = rel.number_of_edges()
        if getattr(rel, "_msg_ind", None) is None:
            rel._msg_ind, rel._msg_frame = np.zeros(m, bool), {}
        for k, t in msgs.items():
            old = rel._msg_frame.get(k)
            if old is None or old.shape[1:] != t.shape[1:]:
                old = t.new_zeros((m,) + tuple(t.shape[1:]))
            rel._msg_frame[k] = old.index_copy(0, st, t)
        rel._msg_ind[sel] = True

    def recv(self, v=ALL, reduce_func=None, apply_node_func=None):
        rel = self._graph
        rfs = _as_list(reduce_func)
        _check_funcs([], rfs)
        vs = np.arange(rel.n_dst) if is_all(v) else np.unique(_ids(v))
        ind = getattr(rel, "_msg_ind", None)
        sel = np.empty(0, np.int64) if ind is None else \
            np.nonzero(ind & np.isin(rel.dst, vs))[0]
        if sel.size == 0:  # scheduler.py:101-107
            if apply_node_func is not None:
                self.apply_nodes(apply_node_func, vs)
            return
        dev = _device_of(self.srcdata, self.dstdata, self.edata)
        st = th.from_numpy(sel).to(dev)
        msgs = {k: t[st] for k, t in rel._msg_frame.items()}
        self._partial(sel, vs, [], rfs, apply_node_func, msgs)
        ind[sel] = False

    def apply_edges(self, func, edges=ALL):
        dev = _device_of(self.srcdata, self.dstdata, self.edata)
        rel = self._graph
        sel = _select(rel, edges)
        m = rel.number_of_edges()
        if sel is None:
            s, d = th.from_numpy(rel.src).to(dev), th.from_numpy(rel.dst).to(dev)
            gidx, ef, k = rel.get_immutable_gidx(dev), self.edata, m
        else:
            s, d = th.from_numpy(rel.src[sel]).to(dev), th.from_numpy(rel.dst[sel]).to(dev)
            gidx = device_block_gidx(rel.n_src, rel.n_dst, s.int(), d.int())
            st = th.from_numpy(sel).to(dev)
            ef, k = {kk: t[st] for kk, t in self.edata.items()}, int(sel.size)
        if isinstance(func, MessageFunction):
            out = {func.out_field: func._invoke(gidx, self.srcdata, self.dstdata, ef, k,
                                                reducer="none")}
        else:
            eb = EdgeBatch(s, d, th.arange(k, device=dev), {kk: t[s] for kk, t in self.srcdata.items()},
                           {kk: t[d] for kk, t in self.dstdata.items()}, dict(ef))
            out = func(eb)
        if sel is None:
            self.edata.update(out)
            return
        st = th.from_numpy(sel).to(dev)
        for kk, t in out.items():
            base = self.edata[kk] if kk in self.edata else t.new_zeros((m,) + tuple(t.shape[1:]))
            self.edata[kk] = base.index_copy(0, st, t.to(base.dtype))


def heterograph(data_dict, num_nodes_dict=None):
    """``dgl.heterograph``: {(srctype, etype, dsttype): (u, v)} -> DGLHeteroGraph."""
    rels, counts = OrderedDict(), OrderedDict()
    for (s, e, d), data in data_dict.items():
        u, v = _uv(data)
        rels[(s, e, d)] = (u, v)
        for t, ids in ((s, u), (d, v)):
            need = int(ids.max()) + 1 if ids.size else 0
            counts[t] = max(counts.get(t, 0), need)
    for t, n in (num_nodes_dict or {}).items():
        counts[t] = int(n)  # explicit sizes win (ids are range-checked by the graph)
    return DGLHeteroGraph(rels, counts)


def graph(data, ntype="_N", etype="_E", num_nodes=None):
    """``dgl.graph``: one node type, one edge type.  ``data`` is (u, v), a list of
    pairs, or a square scipy sparse matrix (rows = source)."""
    if hasattr(data, "tocoo"):
        m = data.tocoo()
        num_nodes = m.shape[0] if num_nodes is None else num_nodes
        data = (m.row, m.col)
    return heterograph({(ntype, etype, ntype): data},
                       None if num_nodes is None else {ntype: num_nodes})


def bipartite(data, utype="_U", etype="_E", vtype="_V", num_nodes=None):
    """``dgl.bipartite``: edges from ``utype`` to ``vtype``.  ``data`` is (u, v),
    a list of pairs, or a scipy sparse matrix (rows = utype, cols = vtype)."""
    sizes = None
    if hasattr(data, "tocoo"):
        m = data.tocoo()
        sizes = {utype: m.shape[0], vtype: m.shape[1]}
        data = (m.row, m.col)
    if num_nodes is not None:
        sizes = {utype: num_nodes[0], vtype: num_nodes[1]}
    return heterograph({(utype, etype, vtype): data}, sizes)


def hetero_from_relations(rel_graphs):
    """``dgl.hetero_from_relations``: one heterograph from single-relation graphs."""
    rels, counts = OrderedDict(), OrderedDict()
    for g in rel_graphs:
        for c in g.canonical_etypes:
            if c in rels:
                raise DGLError("duplicate edge type %s" % (c,))
            r = g._rels[c]
            rels[c] = (r.src, r.dst)
            for t, n in ((c[0], r.n_src), (c[2], r.n_dst)):
                if counts.get(t, n) != n:
                    raise DGLError("node type %s has different sizes in the relations" % t)
                counts[t] = n
    out = DGLHeteroGraph(rels, counts)
    for g in rel_graphs:
        for t in g.ntypes:
            out._nframes[t].update(g._nframes[t])
        for c in g.canonical_etypes:
            out._eframes[c].update(g._eframes[c])
    return out
