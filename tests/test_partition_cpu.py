"""Host partition APIs of the reference (``python/dgl/transform.py:551-630``):
partition_graph_with_halo and metis_partition (METIS replaced; the checks are the
reference's own ``tests/compute/test_transform.py:224-276``), and to_bidirected
(vectorised) against a loop restatement of ``graph_op.cc:332-401``."""
import numpy as np
import pytest

import dgl


def _loop_bidirected(src, dst, n, readonly):
    """graph_op.cc:332-401 restated with loops (ToBidirected{Immutable,Mutable}Graph)."""
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
            seen = []
            for v in preds[u] + succs[u]:
                if v not in seen:
                    seen.append(v)
            for v in seen:
                k = max(cnt.get((u, v), 0), cnt.get((v, u), 0))
                out_s += [v] * k
                out_d += [u] * k
    else:
        for u in range(n):
            for v in range(u, n):
                k = max(cnt.get((u, v), 0), cnt.get((v, u), 0))
                if k == 0:
                    continue
                if u == v:
                    out_s += [u] * k
                    out_d += [u] * k
                else:
                    out_s += [u] * k + [v] * k
                    out_d += [v] * k + [u] * k
    return out_s, out_d


@pytest.mark.parametrize("readonly", [True, False])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_to_bidirected_matches_loop_restatement(readonly, seed):
    rng = np.random.default_rng(seed)
    n = 30
    src = rng.integers(0, n, 120)
    dst = rng.integers(0, n, 120)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    bg = dgl.to_bidirected(g, readonly=readonly)
    s, d = bg.edges()
    es, ed = _loop_bidirected(src, dst, n, readonly)
    assert s.tolist() == es and d.tolist() == ed
    assert bg.is_readonly == readonly


def _random_graph(n, seed=0):
    rng = np.random.default_rng(seed)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(rng.integers(0, n, n * 10), rng.integers(0, n, n * 10))
    return g


def _in_hops(g, nodes, hops):
    """Nodes within `hops` in-hops of `nodes`, and the in-edges of those within hops-1."""
    src, dst = (a.numpy() for a in g.edges())
    reach = set(nodes.tolist())
    frontier = set(reach)
    edges = set()
    for h in range(hops):
        sel = np.isin(dst, list(frontier))
        edges |= set(np.nonzero(sel)[0].tolist())
        new = set(src[sel].tolist()) - reach
        reach |= new
        frontier = new
    return reach, edges


@pytest.mark.parametrize("hops", [1, 2])
def test_partition_with_halo(hops):
    g = _random_graph(300)
    node_part = np.random.default_rng(1).integers(0, 4, g.number_of_nodes())
    subgs = dgl.transform.partition_graph_with_halo(g, node_part, hops)
    assert sorted(subgs) == [0, 1, 2, 3]
    src, dst = (a.numpy() for a in g.edges())
    for pid, sub in subgs.items():
        nodes = np.nonzero(node_part == pid)[0]
        reach, edges = _in_hops(g, nodes, hops)
        assert set(sub.parent_nid.tolist()) == reach
        assert sorted(sub.parent_eid.tolist()) == sorted(edges)
        inner = sub.ndata["inner_node"].numpy()
        assert np.array_equal(sub.parent_nid.numpy()[inner == 1], nodes)
        # subgraph edges are the parent edges, relabelled
        ls, ld = (a.numpy() for a in sub.edges())
        pn, pe = sub.parent_nid.numpy(), sub.parent_eid.numpy()
        assert np.array_equal(pn[ls], src[pe]) and np.array_equal(pn[ld], dst[pe])
        ie = sub.edata["inner_edge"].numpy()
        assert np.array_equal(ie == 1, np.isin(src[pe], nodes) & np.isin(dst[pe], nodes))
        assert sub.is_readonly


def test_metis_partition_structure():
    """tests/compute/test_transform.py:245-274 (the partitioner is LDG here)."""
    g = _random_graph(1000)
    subgs = dgl.transform.metis_partition(g, 4, 0, method="ldg")
    num_inner_nodes = 0
    for part_id, subg in subgs.items():
        assert np.all(subg.ndata["inner_node"].numpy() == 1)
        assert np.all(subg.edata["inner_edge"].numpy() == 1)
        assert np.all(subg.ndata["part_id"].numpy() == part_id)
        num_inner_nodes += subg.number_of_nodes()
    assert num_inner_nodes == g.number_of_nodes()
    subgs = dgl.transform.metis_partition(g, 4, 1, method="ldg")
    num_inner_nodes = 0
    for part_id, subg in subgs.items():
        lnode_ids = np.nonzero(subg.ndata["inner_node"].numpy())[0]
        num_inner_nodes += len(lnode_ids)
        assert np.sum(subg.ndata["part_id"].numpy() == part_id) == len(lnode_ids)
    assert num_inner_nodes == g.number_of_nodes()
