"""Heterograph construction and bookkeeping (host side, no kernels)."""
import pytest
import scipy.sparse as sp

import dgl
from dgl import DGLError


def _g():
    return dgl.heterograph({
        ("user", "follows", "user"): ([0, 1, 2], [1, 2, 0]),
        ("user", "plays", "game"): ([0, 1, 1], [0, 0, 1]),
        ("game", "attracts", "user"): ([1], [2])})


def test_metadata():
    g = _g()
    assert g.ntypes == ["user", "game"]
    assert g.etypes == ["follows", "plays", "attracts"]
    assert g.canonical_etypes[1] == ("user", "plays", "game")
    assert g.number_of_nodes("user") == 3 and g.number_of_nodes("game") == 2
    assert g.number_of_edges("plays") == 3 and g.number_of_edges() == 7
    assert g.to_canonical_etype("attracts") == ("game", "attracts", "user")
    assert g.in_degrees(etype="plays").tolist() == [2, 1]
    assert g.out_degrees(etype="plays").tolist() == [1, 2, 0]
    u, v = g.edges(etype="follows")
    assert u.tolist() == [0, 1, 2] and v.tolist() == [1, 2, 0]
    rel = g["plays"]
    assert rel.number_of_src_nodes() == 3 and rel.number_of_dst_nodes() == 2
    assert g.nodes("game").tolist() == [0, 1]


def test_errors():
    g = _g()
    with pytest.raises(DGLError):
        g.number_of_nodes()          # two node types: must name one
    with pytest.raises(DGLError):
        g.to_canonical_etype("nope")
    with pytest.raises(DGLError):
        dgl.heterograph({("a", "r", "b"): ([0, 5], [0, 1])}, {"a": 2, "b": 2})  # id out of range
    with pytest.raises(DGLError):
        g["plays"].ndata            # bipartite: ndata is ambiguous


def test_constructors():
    g1 = dgl.graph([(0, 1), (1, 1)], "user", "follows")
    g2 = dgl.bipartite([(0, 1)], "game", "attracts", "user")
    g = dgl.hetero_from_relations([g1, g2])
    assert g.canonical_etypes == [("user", "follows", "user"), ("game", "attracts", "user")]
    assert g.number_of_nodes("user") == 2 and g.number_of_nodes("game") == 1
    m = sp.random(5, 7, density=0.3, random_state=0, format="csr")
    b = dgl.bipartite(m, "u", "r", "v")
    assert b.number_of_nodes("u") == 5 and b.number_of_nodes("v") == 7
    assert b.number_of_edges() == m.nnz
    single = dgl.graph(([0, 1], [1, 2]), num_nodes=5)
    assert single.number_of_nodes() == 5 and single.number_of_edges() == 2


def test_local_scope_isolates_frames():
    import torch as th
    g = _g()
    g.nodes["user"].data["h"] = th.zeros(3)
    with g.local_scope():
        g.nodes["user"].data["h"] = th.ones(3)
        g.nodes["user"].data["tmp"] = th.ones(3)
    assert g.nodes["user"].data["h"].sum() == 0 and "tmp" not in g.nodes["user"].data
    lv = g["follows"].local_var()
    lv.srcdata["x"] = th.ones(3)
    assert "x" not in g.nodes["user"].data
