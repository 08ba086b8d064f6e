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
    each way (``graph_op.cc:332-401``), vectorised.  Edge order as the
    reference's general paths: readonly (``ToBidirectedImmutableGraph``) -- for
    each node u, its distinct neighbours (predecessors, then successors, in
    edge-id order), each v contributing v->u; mutable (``ToBidirectedMutableGraph``)
    -- for u <= v, the u->v copies then the v->u copies.  The reference tries a
    GKlib symmetric-CSR path first for readonly INPUT graphs
    (``graph_op.cc:651-654``); its edge order is not reproduced (parity unpinned
    for that case).  ``readonly=True`` returns a readonly graph."""
    src, dst = _coo(g)
    n = g.number_of_nodes()
    keys, counts = np.unique(src * n + dst, return_counts=True)

    def count(u, v):  # number of u -> v edges
        k = u * n + v
        pos = np.searchsorted(keys, k)
        pos_c = np.minimum(pos, max(len(keys) - 1, 0))
        hit = (pos < len(keys)) & (keys[pos_c] == k) if len(keys) else np.zeros(len(k), bool)
        return np.where(hit, counts[pos_c] if len(keys) else 0, 0)

    if readonly:
        m = len(src)
        # per node u: predecessors (phase 0) then successors (phase 1), edge-id order
        u = np.concatenate([dst, src])
        v = np.concatenate([src, dst])
        order = np.lexsort((np.arange(2 * m), np.repeat([0, 1], m), u))
        u, v = u[order], v[order]
        _, first = np.unique(u * n + v, return_index=True)
        first.sort()
        u, v = u[first], v[first]
        k = np.maximum(count(u, v), count(v, u))
        out_s, out_d = np.repeat(v, k), np.repeat(u, k)
    else:
        a, b = np.minimum(src, dst), np.maximum(src, dst)
        pairs = np.unique(a * n + b)
        u, v = pairs // n, pairs % n
        k = np.maximum(count(u, v), count(v, u))
        reps = np.where(u == v, k, 2 * k)
        pid = np.repeat(np.arange(len(u)), reps)
        j = np.arange(int(reps.sum())) - np.repeat(np.cumsum(reps) - reps, reps)
        first_half = j < k[pid]
        out_s = np.where(first_half, u[pid], v[pid])
        out_d = np.where(first_half, v[pid], u[pid])
    bg = _new_graph(n, out_s, out_d)
    bg._readonly = bool(readonly)
    return bg


def partition_graph_with_halo(g, node_part, num_hops):
    """Partition ``g`` by ``node_part`` into subgraphs that carry their halo
    (``transform.py:551-587``, ``_CAPI_DGLPartitionWithHalo`` /
    ``GraphOp::GetSubgraphWithHalo``, ``graph_op.cc:403-509``): partition p holds
    its nodes, their in-edges (only those from inner nodes when ``num_hops`` is 0)
    and, hop by hop, the in-edges of the nodes reached so far, up to ``num_hops``.
    Node ids keep the parent order (ascending); edges are listed as the reference
    collects them (in-edges of the inner nodes, then of each hop's new nodes, in
    in-CSR order).  Each subgraph is a readonly DGLGraph with ``parent_nid``,
    ``parent_eid``, ``ndata['inner_node']`` and ``edata['inner_edge']`` (int32).
    Host-side setup, as in the reference."""
    import torch as th
    from .graph import DGLGraph
    node_part = np.asarray(node_part.cpu() if hasattr(node_part, "cpu") else node_part,
                           dtype=np.int64)
    n = g.number_of_nodes()
    if node_part.shape[0] != n:
        raise ValueError("node_part needs one entry per node")
    _, in_csr = g._graph.host_csr()
    indptr, indices, eids = in_csr

    def in_edges(vs):
        beg, end = indptr[vs], indptr[vs + 1]
        lens = end - beg
        pos = np.repeat(beg - np.cumsum(lens) + lens, lens) + np.arange(int(lens.sum()))
        return indices[pos], np.repeat(vs, lens), eids[pos]

    out = {}
    for p in np.unique(node_part):
        nodes = np.nonzero(node_part == p)[0]
        seen = np.zeros(n, bool)
        seen[nodes] = True
        s, d, e = in_edges(nodes)
        inner_e = seen[s]
        if num_hops == 0:
            s, d, e, inner_e = s[inner_e], d[inner_e], e[inner_e], inner_e[inner_e]
        srcs, dsts, es, inn = [s], [d], [e], [inner_e]
        frontier = None
        if num_hops > 0:
            _, first = np.unique(s, return_index=True)
            cand = s[np.sort(first)]
            frontier = cand[~seen[cand]]
            seen[frontier] = True
        for _ in range(1, num_hops):
            s, d, e = in_edges(frontier)
            srcs.append(s)
            dsts.append(d)
            es.append(e)
            inn.append(np.zeros(len(s), bool))
            _, first = np.unique(s, return_index=True)
            cand = s[np.sort(first)]
            frontier = cand[~seen[cand]]
            seen[frontier] = True
        old_ids = np.nonzero(seen)[0]
        new_of = np.full(n, -1, np.int64)
        new_of[old_ids] = np.arange(len(old_ids))
        s, d = np.concatenate(srcs), np.concatenate(dsts)
        sub = _new_graph(len(old_ids), new_of[s], new_of[d])
        sub._readonly = True
        sub.parent_nid = th.from_numpy(old_ids)
        sub.parent_eid = th.from_numpy(np.concatenate(es))
        sub.ndata["inner_node"] = th.from_numpy((node_part[old_ids] == p).astype(np.int32))
        sub.edata["inner_edge"] = th.from_numpy(np.concatenate(inn).astype(np.int32))
        out[int(p)] = sub
    return out


def metis_partition(g, k, extra_cached_hops=0, method=None):
    """``dgl.transform.metis_partition`` (``transform.py:589-630``): a k-way node
    partition of the symmetrised graph, then :func:`partition_graph_with_halo`;
    every subgraph gets ``ndata['part_id']``.  METIS (``metis_partition.cc:19-66``)
    is absent here: the partition comes from the device label propagation
    (``dgl.distributed.partition_labelprop``, balanced by node count like METIS's
    default) when a GPU is present, else from the native LDG
    (``DGLMIPartitionLDG``).  ``method`` ("labelprop" | "ldg") forces one."""
    import torch as th
    from . import distributed as D
    src, dst = _coo(g)
    n = g.number_of_nodes()
    if method is None:
        method = "labelprop" if th.cuda.is_available() else "ldg"
    if k == 1:
        part = np.zeros(n, np.int64)
    elif method == "labelprop":
        from .graph_index import device_block_gidx
        dev = th.device("cuda", th.cuda.current_device())
        gidx = device_block_gidx(n, n, th.as_tensor(src, dtype=th.int32, device=dev),
                                 th.as_tensor(dst, dtype=th.int32, device=dev))
        a, _ = D.partition_labelprop(gidx, k, balance="nodes", slack=0.03)
        part = a.cpu().numpy().astype(np.int64)
    elif method == "ldg":
        part = D.partition_ldg(n, src, dst, k, slack=0.03)
    else:
        raise ValueError("unknown partition method %s" % method)
    parts = partition_graph_with_halo(g, part, extra_cached_hops)
    for pid, sub in parts.items():
        sub.ndata["part_id"] = th.from_numpy(part[sub.parent_nid.numpy()])
    return parts
