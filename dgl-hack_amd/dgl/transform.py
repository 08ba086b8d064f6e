"""Graph transforms used by the conv modules (``python/dgl/transform.py``)."""
import numpy as np


def laplacian_lambda_max(g):
    """Largest eigenvalue of I - D^-1/2 A D^-1/2 (in-degree norm, clipped at 1) per
    graph, as a list (``transform.py:396-434``; an unbatched graph is a batch of
    one).  Host scipy ``eigs`` as the reference -- setup work, not on the
    message-passing path."""
    from scipy import sparse
    from scipy.sparse import linalg
    n = g.number_of_nodes()
    adj = g.adjacency_matrix_scipy().astype(float)
    deg = np.asarray(g.in_degrees().numpy(), dtype=float).clip(1)
    norm = sparse.diags(deg ** -0.5, dtype=float)
    lap = sparse.eye(n) - norm * adj * norm
    return [float(linalg.eigs(lap, 1, which="LM", return_eigenvectors=False)[0].real)]


def _new_graph(n, src, dst):
    from .graph import DGLGraph
    g = DGLGraph()
    g.add_nodes(n)
    if len(src):
        g.add_edges(np.asarray(src, dtype=np.int64), np.asarray(dst, dtype=np.int64))
    return g


def _coo(g):
    src, dst, _ = g._graph.edges()
    return np.asarray(src, dtype=np.int64), np.asarray(dst, dtype=np.int64)


def add_self_loop(g):
    """Existing self-loops dropped, then one self-loop per node appended, edges kept
    in id order (``transform.py:486-519``)."""
    src, dst = _coo(g)
    keep = src != dst
    nodes = np.arange(g.number_of_nodes(), dtype=np.int64)
    return _new_graph(g.number_of_nodes(), np.concatenate([src[keep], nodes]),
                      np.concatenate([dst[keep], nodes]))


def remove_self_loop(g):
    """``transform.py:521-549``."""
    src, dst = _coo(g)
    keep = src != dst
    return _new_graph(g.number_of_nodes(), src[keep], dst[keep])


def reverse(g, share_ndata=False, share_edata=False):
    """Edges reversed, same ids (``transform.py:258-335``); ``share_*`` shares the
    feature frames with ``g``."""
    src, dst = _coo(g)
    rg = _new_graph(g.number_of_nodes(), dst, src)
    if share_ndata:
        rg._node_frame = g._node_frame
    if share_edata:
        rg._edge_frame = g._edge_frame
    return rg


def to_bidirected(g, readonly=True):
    """Both directions of every edge; a pair (u, v) gets max(#u->v, #v->u) edges
    each way (``graph_op.cc:332-401``).  Edge order as the reference: readonly --
    for each node u, its distinct neighbours (predecessors, then successors, in
    edge-id order), each v contributing v->u; mutable -- for u <= v, the u->v
    copies then the v->u copies."""
    src, dst = _coo(g)
    n = g.number_of_nodes()
    cnt = {}
    for u, v in zip(src.tolist(), dst.tolist()):
        cnt[(u, v)] = cnt.get((u, v), 0) + 1
    out_s, out_d = [], []
    if readonly:
        preds = [[] for _ in range(n)]
        succs = [[] for _ in range(n)]
        for u, v in zip(src.tolist(), dst.tolist()):
            preds[v].append(u)
            succs[u].append(v)
        for u in range(n):
            seen = set()
            for v in preds[u] + succs[u]:
                if v in seen:
                    continue
                seen.add(v)
                k = max(cnt.get((u, v), 0), cnt.get((v, u), 0))
                out_s += [v] * k
                out_d += [u] * k
    else:
        pairs = sorted({(min(u, v), max(u, v)) for (u, v) in cnt})
        for u, v in pairs:
            k = max(cnt.get((u, v), 0), cnt.get((v, u), 0))
            if u == v:
                out_s += [u] * k
                out_d += [u] * k
            else:
                out_s += [u] * k + [v] * k
                out_d += [v] * k + [u] * k
    return _new_graph(n, out_s, out_d)
