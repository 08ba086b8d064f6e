"""Host-side checks for the conv-module zoo (no GPU): the Laplacian eigenvalue
known answer (``python/dgl/transform.py:418-423`` docstring), module
construction / parameter shapes / aggregator validation as the reference
modules, and that a CPU tensor is refused (the engine has no CPU path)."""
import pytest
import scipy as sp
import scipy.sparse  # noqa: F401
import torch as th

import dgl
import dgl.nn.pytorch as nn


def test_laplacian_lambda_max_known_answer():
    g = dgl.DGLGraph()
    g.add_nodes(5)
    g.add_edges([0, 1, 2, 3, 4, 0, 1, 2, 3, 4], [1, 2, 3, 4, 0, 4, 0, 1, 2, 3])
    lam = dgl.laplacian_lambda_max(g)
    assert len(lam) == 1 and abs(lam[0] - 1.809016994374948) < 1e-9


def test_graph_from_scipy():
    m = sp.sparse.random(50, 50, density=0.1, random_state=0)
    g = dgl.graph(m)
    assert g.number_of_nodes() == 50 and g.number_of_edges() == m.nnz and g.is_homograph()
    assert g.number_of_src_nodes() == g.number_of_dst_nodes() == 50


@pytest.mark.parametrize("ctor,params", [
    (lambda: nn.SAGEConv(5, 10, "mean"), {"fc_self.weight": (10, 5), "fc_neigh.weight": (10, 5)}),
    (lambda: nn.SAGEConv(5, 10, "gcn"), {"fc_neigh.weight": (10, 5)}),
    (lambda: nn.SAGEConv(5, 10, "pool"), {"fc_pool.weight": (5, 5)}),
    (lambda: nn.SGConv(5, 10, 3), {"fc.weight": (10, 5)}),
    (lambda: nn.TAGConv(5, 2, k=2), {"lin.weight": (2, 15)}),
    (lambda: nn.ChebConv(5, 2, 3), {"fc.2.weight": (2, 5), "bias": (2,)}),
    (lambda: nn.EdgeConv(5, 2), {"theta.weight": (2, 5), "phi.weight": (2, 5)}),
    (lambda: nn.GatedGraphConv(5, 10, 5, 3), {"linears.2.weight": (10, 10),
                                              "gru.weight_ih": (30, 10)}),
    (lambda: nn.AGNNConv(1), {"beta": (1,)}),
])
def test_module_parameters(ctor, params):
    named = dict(ctor().named_parameters())
    for k, shp in params.items():
        assert tuple(named[k].shape) == shp


def test_bad_aggregators():
    for ctor in (lambda: nn.SAGEConv(5, 10, "median"), lambda: nn.GINConv(None, "prod")):
        with pytest.raises(KeyError):
            ctor()


def test_cpu_tensors_refused():
    g = dgl.DGLGraph()
    g.add_nodes(4)
    g.add_edges([0, 1, 2], [1, 2, 3])
    for m, args in ((nn.SAGEConv(3, 2, "mean"), (th.randn(4, 3),)),
                    (nn.GINConv(None, "sum"), (th.randn(4, 3),)),
                    (nn.SGConv(3, 2), (th.randn(4, 3),)),
                    (nn.EdgeConv(3, 2), (th.randn(4, 3),))):
        with pytest.raises(Exception):
            m(g, *args)


def test_adjacency_orientation():
    """DGL 0.4: a row of adjacency_matrix() is a destination (graph.py:3567-3599)."""
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 0], [1, 2])
    a = g.adjacency_matrix().to_dense()
    assert a[1, 0] == 1 and a[2, 0] == 1 and a[0, 1] == 0
    assert (g.adjacency_matrix(transpose=True).to_dense() == a.t()).all()
    assert (g.adjacency_matrix_scipy().toarray() == a.numpy()).all()
    b = dgl.bipartite(([0, 1], [2, 0]), num_nodes=(2, 3))
    ab = b.adjacency_matrix().to_dense()
    assert ab.shape == (3, 2) and ab[2, 0] == 1 and ab[0, 1] == 1


def test_dense_modules_on_host():
    """The dense modules are plain torch (GEMMs): they run anywhere."""
    adj = (th.rand(30, 30) < 0.2).float()
    x = th.randn(30, 4)
    assert nn.DenseGraphConv(4, 3)(adj, x).shape == (30, 3)
    assert nn.DenseSAGEConv(4, 3)(adj, x).shape == (30, 3)
    assert nn.DenseChebConv(4, 3, 3)(adj, x).shape == (30, 3)


def test_transform_known_answers():
    """Docstring known answers of transform.py: add_self_loop (:497-503),
    to_bidirected (:371-378), reverse (:270-290), remove_self_loop."""
    g = dgl.DGLGraph()
    g.add_nodes(5)
    g.add_edges([0, 1, 2], [1, 1, 2])
    s, d = dgl.transform.add_self_loop(g).edges()
    assert s.tolist() == [0, 0, 1, 2, 3, 4] and d.tolist() == [1, 0, 1, 2, 3, 4]
    s, d = dgl.remove_self_loop(g).edges()
    assert s.tolist() == [0] and d.tolist() == [1]
    g = dgl.DGLGraph()
    g.add_nodes(2)
    g.add_edges([0, 0], [0, 1])
    s, d = dgl.to_bidirected(g).edges()
    assert s.tolist() == [0, 1, 0] and d.tolist() == [0, 0, 1]
    s, d = dgl.to_bidirected(g, readonly=False).edges()
    assert sorted(zip(s.tolist(), d.tolist())) == [(0, 0), (0, 1), (1, 0)]
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 1, 2], [1, 2, 0])
    g.ndata["h"] = th.tensor([[0.], [1.], [2.]])
    rg = g.reverse(share_ndata=True)
    s, d = rg.edges()
    assert s.tolist() == [1, 2, 0] and d.tolist() == [0, 1, 2]
    assert th.equal(rg.ndata["h"], g.ndata["h"])
    # multigraph: max of the two directions' multiplicities
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 0, 1, 2], [1, 1, 0, 2])
    s, d = dgl.to_bidirected(g).edges()
    pairs = sorted(zip(s.tolist(), d.tolist()))
    assert pairs == [(0, 1), (0, 1), (1, 0), (1, 0), (2, 2)]
