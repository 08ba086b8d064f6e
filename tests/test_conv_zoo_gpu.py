"""The remaining dgl.nn.pytorch conv modules (SAGE, GIN, SG, APPNP, TAG, Cheb,
AGNN, EdgeConv, GatedGraph) on the HIP path.

Each module is checked three ways: against a dense float64 restatement of the
reference's formula (its forward in ``python/dgl/nn/pytorch/conv/*.py``),
forward and gradients; where it has a fused MI355X form, against its own
``fused = False`` reference-order path (update_all builtins / UDFs); and the
reference's own tests (``tests/pytorch/test_nn.py:100-132, 426-595, 634-665,
733-747``) for shapes, caching and the TAGConv / Cheb known answers.
Tolerance: 1e-4 relative / absolute (fp32 aggregation, north_star).
"""
import copy

import networkx as nx
import numpy as np
import pytest
import scipy as sp
import scipy.sparse  # noqa: F401
import torch as th

import dgl
import dgl.nn.pytorch as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = dict(rtol=1e-4, atol=1e-4)


def _rand_graph(n=300, m=3000, seed=0, self_loops=False):
    rng = np.random.default_rng(seed)
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    if self_loops:
        src, dst = np.concatenate([src, np.arange(n)]), np.concatenate([dst, np.arange(n)])
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g


def _bipartite(n_src=100, n_dst=200, m=2000, seed=1):
    rng = np.random.default_rng(seed)
    src = np.concatenate([rng.integers(0, n_src, m), rng.integers(0, n_src, n_dst)])
    dst = np.concatenate([rng.integers(0, n_dst, m), np.arange(n_dst)])  # every dst has an edge
    return dgl.bipartite((src, dst), num_nodes=(n_src, n_dst))


def _edges(g):
    s, d, _ = g._graph.edges()
    return th.as_tensor(np.asarray(s)), th.as_tensor(np.asarray(d))


def _adj(g):
    """Dense (n_dst, n_src) float64 adjacency, duplicate edges counted."""
    s, d = _edges(g)
    n_src = g.number_of_src_nodes() if hasattr(g, "number_of_src_nodes") else g.number_of_nodes()
    n_dst = g.number_of_dst_nodes() if hasattr(g, "number_of_dst_nodes") else g.number_of_nodes()
    A = th.zeros(n_dst, n_src, dtype=th.float64)
    A.index_put_((d, s), th.ones(len(s), dtype=th.float64), accumulate=True)
    return A.to(DEV)


def _grads(module, *inputs):
    return [p.grad.clone() for p in module.parameters() if p.grad is not None] + \
        [x.grad.clone() for x in inputs if x.grad is not None]


def _run(module, g, *inputs):
    module.zero_grad()
    for x in inputs:
        if isinstance(x, th.Tensor) and x.grad is not None:
            x.grad = None
    out = module(g, *inputs)
    (out * th.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
    return out.detach(), _grads(module, *[x for x in inputs if isinstance(x, th.Tensor)])


def _fused_vs_reference(module, g, *inputs):
    """Forward + every gradient of the fused form vs fused = False."""
    module.fused = True
    out_f, gr_f = _run(module, g, *inputs)
    module.fused = False
    out_r, gr_r = _run(module, g, *inputs)
    module.fused = True
    assert th.allclose(out_f, out_r, **TOL), (out_f - out_r).abs().max()
    assert len(gr_f) == len(gr_r)
    for a, b in zip(gr_f, gr_r):
        assert th.allclose(a, b, **TOL), (a - b).abs().max()
    return out_f


def _lin64(lin, x):
    y = x @ lin.weight.detach().double().t()
    return y if lin.bias is None else y + lin.bias.detach().double()


# ------------------------------------------------------------------------- SAGE
@pytest.mark.parametrize("aggre", ["mean", "gcn", "pool"])
@pytest.mark.parametrize("fin,fout", [(32, 8), (8, 32)])
def test_sage_conv_dense(aggre, fin, fout):
    g = _rand_graph(self_loops=True)
    th.manual_seed(0)
    sage = nn.SAGEConv(fin, fout, aggre).to(DEV)
    x = th.randn(g.number_of_nodes(), fin, device=DEV, requires_grad=True)
    out = _fused_vs_reference(sage, g, x) if aggre != "pool" else sage(g, x)
    A = _adj(g)
    xd = x.detach().double()
    deg = A.sum(1, keepdim=True)
    if aggre == "mean":
        neigh = (A @ xd) / deg.clamp(min=1)
    elif aggre == "gcn":
        neigh = (A @ xd + xd) / (deg + 1)
    else:
        hp = th.relu(_lin64(sage.fc_pool, xd))
        big = th.where(A[:, :, None] > 0, hp[None, :, :], th.tensor(-np.inf, device=DEV, dtype=th.float64))
        neigh = big.max(1).values
    want = _lin64(sage.fc_neigh, neigh)
    if aggre != "gcn":
        want = _lin64(sage.fc_self, xd) + want
    assert th.allclose(out.double(), want, **TOL), (out.double() - want).abs().max()


@pytest.mark.parametrize("aggre", ["mean", "gcn", "pool", "lstm"])
def test_sage_conv_reference_shapes(aggre):
    """test_nn.py:426-449 (readonly DGLGraph, dgl.graph, dgl.bipartite)."""
    th.manual_seed(0)
    g = dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1), readonly=True)
    sage = nn.SAGEConv(5, 10, aggre).to(DEV)
    assert sage(g, th.randn(100, 5, device=DEV)).shape[-1] == 10
    g = dgl.graph(sp.sparse.random(100, 100, density=0.1))
    if aggre != "lstm":  # UDF reducers run on DGLGraph (degree bucketing)
        sage = nn.SAGEConv(5, 10, aggre).to(DEV)
        assert sage(g, th.randn(100, 5, device=DEV)).shape[-1] == 10
        g = dgl.bipartite(sp.sparse.random(100, 200, density=0.1))
        dst_dim = 5 if aggre != "gcn" else 10
        sage = nn.SAGEConv((10, dst_dim), 2, aggre).to(DEV)
        h = sage(g, (th.randn(100, 10, device=DEV), th.randn(200, dst_dim, device=DEV)))
        assert h.shape == (200, 2)


def test_sage_bipartite_fused():
    g = _bipartite()
    th.manual_seed(0)
    for aggre in ("mean", "gcn"):
        sage = nn.SAGEConv((16, 16), 4, aggre).to(DEV)
        xs = th.randn(100, 16, device=DEV, requires_grad=True)
        xd = th.randn(200, 16, device=DEV, requires_grad=True)
        out = _fused_vs_reference(sage, g, (xs, xd))
        assert out.shape == (200, 4)


def test_sage_lstm_udf_reducer():
    g = _rand_graph(n=60, m=400, self_loops=True)
    th.manual_seed(0)
    sage = nn.SAGEConv(6, 3, "lstm").to(DEV)
    x = th.randn(60, 6, device=DEV, requires_grad=True)
    out = sage(g, x)
    out.sum().backward()
    assert out.shape == (60, 3) and th.isfinite(out).all() and x.grad is not None


# ------------------------------------------------------------------------- GIN
@pytest.mark.parametrize("aggre", ["sum", "mean", "max"])
def test_gin_conv_dense(aggre):
    g = _rand_graph(self_loops=True)
    th.manual_seed(0)
    gin = nn.GINConv(th.nn.Linear(16, 12), aggre, init_eps=0.3, learn_eps=True).to(DEV)
    x = th.randn(g.number_of_nodes(), 16, device=DEV, requires_grad=True)
    out = _fused_vs_reference(gin, g, x) if aggre != "max" else gin(g, x)
    A, xd = _adj(g), x.detach().double()
    if aggre == "sum":
        neigh = A @ xd
    elif aggre == "mean":
        neigh = (A @ xd) / A.sum(1, keepdim=True).clamp(min=1)
    else:
        neigh = th.where(A[:, :, None] > 0, xd[None], th.tensor(-np.inf, device=DEV,
                                                                dtype=th.float64)).max(1).values
    want = _lin64(gin.apply_func, (1 + gin.eps.detach().double()) * xd + neigh)
    assert th.allclose(out.double(), want, **TOL)


@pytest.mark.parametrize("aggre", ["mean", "max", "sum"])
def test_gin_conv_reference_shapes(aggre):
    """test_nn.py:481-501."""
    g = dgl.graph(sp.sparse.random(100, 100, density=0.1))
    gin = nn.GINConv(th.nn.Linear(5, 12), aggre).to(DEV)
    assert gin(g, th.randn(100, 5, device=DEV)).shape == (100, 12)
    g = dgl.bipartite(sp.sparse.random(100, 200, density=0.1))
    gin = nn.GINConv(th.nn.Linear(5, 12), aggre).to(DEV)
    h = gin(g, (th.randn(100, 5, device=DEV), th.randn(200, 5, device=DEV)))
    assert h.shape == (200, 12)


# ------------------------------------------------------------- SG / APPNP / TAG
def _sym(g):
    A = _adj(g)
    norm = A.sum(1).clamp(min=1).pow(-0.5)
    return A, norm[:, None]


def test_sgconv_dense_and_cache():
    g = _rand_graph()
    th.manual_seed(0)
    sgc = nn.SGConv(16, 10, k=3).to(DEV)
    x = th.randn(g.number_of_nodes(), 16, device=DEV, requires_grad=True)
    out = _fused_vs_reference(sgc, g, x)
    A, nrm = _sym(g)
    h = x.detach().double()
    for _ in range(3):
        h = nrm * (A @ (nrm * h))
    assert th.allclose(out.double(), _lin64(sgc.fc, h), **TOL)
    # test_nn.py:451-468: cached features ignore the new input
    sgc = nn.SGConv(5, 10, 3, True).to(DEV)
    gr = dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1), readonly=True)
    f = th.randn(100, 5, device=DEV)
    h0, h1 = sgc(gr, f), sgc(gr, f + 1)
    assert th.allclose(h0, h1) and h0.shape[-1] == 10


@pytest.mark.parametrize("edge_drop", [0.0, 0.3])
def test_appnp_dense(edge_drop):
    g = _rand_graph()
    th.manual_seed(0)
    appnp = nn.APPNPConv(10, 0.1, edge_drop=edge_drop).to(DEV).eval()
    x = th.randn(g.number_of_nodes(), 5, device=DEV, requires_grad=True)
    out = _fused_vs_reference(appnp, g, x)
    A, nrm = _sym(g)
    x0 = h = x.detach().double()
    for _ in range(10):
        h = 0.9 * nrm * (A @ (nrm * h)) + 0.1 * x0
    assert th.allclose(out.double(), h, **TOL)
    if edge_drop > 0:  # training with edge dropout: the u_mul_e path, shape only
        appnp.train()
        assert appnp(g, x).shape == (g.number_of_nodes(), 5)


def test_tagconv_known_answer():
    """test_nn.py:100-132: TAGConv on path_graph(3) == [X, SAS X, (SAS)^2 X] W + b."""
    g = dgl.DGLGraph(nx.path_graph(3))
    A = _adj(g).float()
    norm = th.pow(th.from_numpy(g.in_degrees().numpy()).float(), -0.5).to(DEV)[:, None]
    conv = nn.TAGConv(5, 2, bias=True).to(DEV)
    h0 = th.ones(3, 5, device=DEV)
    h1 = conv(g, h0)
    assert len(g.ndata) == 0 and len(g.edata) == 0
    x1 = (A @ (h0 * norm)) * norm
    x2 = (A @ (x1 * norm)) * norm
    want = th.cat([h0, x1, x2], -1) @ conv.lin.weight.t() + conv.lin.bias
    assert th.allclose(h1, want, **TOL)
    old = copy.deepcopy(conv.lin.weight.data)
    conv.reset_parameters()
    assert not th.allclose(old, conv.lin.weight.data)


def test_tagconv_fused():
    g = _rand_graph()
    th.manual_seed(0)
    conv = nn.TAGConv(8, 6, k=3).to(DEV)
    x = th.randn(g.number_of_nodes(), 8, device=DEV, requires_grad=True)
    _fused_vs_reference(conv, g, x)


# ------------------------------------------------------------------------- Cheb
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_cheb_conv_dense(k):
    """test_nn.py:649-665 restated: ChebConv == the dense Chebyshev recurrence
    on L_hat = 2 L / lambda - I, L = I - D^-1/2 A D^-1/2."""
    g = dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1, random_state=3), readonly=True)
    th.manual_seed(k)
    cheb = nn.ChebConv(5, 2, k).to(DEV)
    x = th.randn(100, 5, device=DEV, requires_grad=True)
    out = _fused_vs_reference(cheb, g, x, [2.0])
    A, nrm = _sym(g)
    L = th.eye(100, dtype=th.float64, device=DEV) - nrm * A * nrm.t()
    Lh = 2.0 * L / 2.0 - th.eye(100, dtype=th.float64, device=DEV)
    t0 = x.detach().double()
    ts = [t0]
    if k > 1:
        ts.append(Lh @ t0)
    for _ in range(2, k):
        ts.append(2 * Lh @ ts[-1] - ts[-2])
    want = sum(t @ cheb.fc[i].weight.detach().double().t() for i, t in enumerate(ts))
    want = want + cheb.bias.detach().double()
    assert th.allclose(out.double(), want, **TOL)


def test_cheb_conv_lambda_default():
    g = _rand_graph(n=80, m=600, seed=4)
    th.manual_seed(0)
    cheb = nn.ChebConv(4, 3, 3).to(DEV)
    x = th.randn(80, 4, device=DEV)
    lam = dgl.laplacian_lambda_max(g)
    assert th.allclose(cheb(g, x), cheb(g, x, lam), **TOL)


# ------------------------------------------------------------------------- AGNN
def test_agnn_conv_dense():
    g = _rand_graph(self_loops=True)
    th.manual_seed(0)
    agnn = nn.AGNNConv(init_beta=1.5).to(DEV)
    x = th.randn(g.number_of_nodes(), 8, device=DEV, requires_grad=True)
    out = agnn(g, x)
    out.sum().backward()
    s, d = _edges(g)
    s, d = s.to(DEV), d.to(DEV)
    xd = x.detach().double()
    nh = xd / xd.norm(dim=1, keepdim=True).clamp(min=1e-12)
    e = 1.5 * (nh[s] * nh[d]).sum(1)
    emax = th.full((g.number_of_nodes(),), -np.inf, dtype=th.float64, device=DEV)
    emax = emax.scatter_reduce(0, d, e, "amax")
    p = th.exp(e - emax[d])
    den = th.zeros(g.number_of_nodes(), dtype=th.float64, device=DEV).index_add_(0, d, p)
    a = p / den[d]
    want = th.zeros_like(xd).index_add_(0, d, a[:, None] * xd[s])
    assert th.allclose(out.double(), want, **TOL)
    assert agnn.beta.grad is not None and x.grad is not None


def test_agnn_reference_shapes():
    """test_nn.py:503-517."""
    g = dgl.graph(sp.sparse.random(100, 100, density=0.1))
    agnn = nn.AGNNConv(1).to(DEV)
    assert agnn(g, th.randn(100, 5, device=DEV)).shape == (100, 5)


# --------------------------------------------------------------------- EdgeConv
def test_edge_conv_fused_dense():
    g = _rand_graph(self_loops=True)
    th.manual_seed(0)
    conv = nn.EdgeConv(6, 4).to(DEV)
    x = th.randn(g.number_of_nodes(), 6, device=DEV, requires_grad=True)
    out = _fused_vs_reference(conv, g, x)
    s, d = _edges(g)
    xd = x.detach().double()
    e = _lin64(conv.theta, xd[d] - xd[s]) + _lin64(conv.phi, xd[s])
    want = th.full((g.number_of_nodes(), 4), -np.inf, dtype=th.float64, device=DEV)
    want = want.scatter_reduce(0, d.to(DEV)[:, None].expand(-1, 4), e, "amax")
    assert th.allclose(out.double(), want, **TOL)


@pytest.mark.parametrize("case", ["ties", "zero_in_degree"])
def test_edge_conv_fused_ties(case):
    """The reference's max gradient reaches every tied edge: repeated feature
    values (many exact ties per destination) and destinations with no in-edge
    (identity output, no gradient)."""
    g = _rand_graph(n=200, m=600, seed=6, self_loops=(case == "ties"))
    th.manual_seed(0)
    conv = nn.EdgeConv(6, 4).to(DEV)
    if case == "ties":
        x = th.randint(0, 2, (200, 6), device=DEV).float().requires_grad_()
    else:
        x = th.randn(200, 6, device=DEV, requires_grad=True)
        assert (th.from_numpy(g.in_degrees().numpy()) == 0).any()
    _fused_vs_reference(conv, g, x)


def test_edge_conv_reference_cases():
    """test_nn.py:634-647 (homogeneous and bipartite) and the batch-norm form."""
    g = _rand_graph(n=20, m=80, seed=5, self_loops=True)
    conv = nn.EdgeConv(5, 2).to(DEV)
    assert conv(g, th.randn(20, 5, device=DEV)).shape == (20, 2)
    gb = _bipartite(20, 10, 60)
    h0 = th.randn(20, 5, device=DEV)
    assert conv(gb, (h0, h0[:10])).shape == (10, 2)
    bn = nn.EdgeConv(5, 2, batch_norm=True).to(DEV)
    assert bn(g, th.randn(20, 5, device=DEV)).shape == (20, 2)


# ------------------------------------------------------------------ GatedGraph
def test_gated_graph_conv_fused_dense():
    g = _rand_graph(n=150, m=1200, seed=2)
    th.manual_seed(0)
    conv = nn.GatedGraphConv(5, 10, 3, 4).to(DEV)
    etypes = (th.arange(g.number_of_edges()) % 4).to(DEV)
    x = th.randn(150, 5, device=DEV, requires_grad=True)
    out = _fused_vs_reference(conv, g, x, etypes)
    s, d = _edges(g)
    s, d, et = s.to(DEV), d.to(DEV), etypes
    h = th.cat([x.detach().double(), th.zeros(150, 5, dtype=th.float64, device=DEV)], 1)
    gru = copy.deepcopy(conv.gru).double()
    for _ in range(3):
        msg = th.zeros(len(s), 10, dtype=th.float64, device=DEV)
        for t in range(4):
            sel = et == t
            msg[sel] = _lin64(conv.linears[t], h[s[sel]])
        a = th.zeros(150, 10, dtype=th.float64, device=DEV).index_add_(0, d, msg)
        h = gru(a, h)
    assert th.allclose(out.double(), h.detach(), **TOL)


def test_gated_graph_reference_shape():
    """test_nn.py:519-530."""
    g = dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1), readonly=True)
    conv = nn.GatedGraphConv(5, 10, 5, 3).to(DEV)
    etypes = (th.arange(g.number_of_edges()) % 3).to(DEV)
    assert conv(g, th.randn(100, 5, device=DEV), etypes).shape[-1] == 10


def test_builtins_only_reach_hip():
    """The fused modules really run the engine's copy_u_sum kernel: a graph on a
    non-ROCm device is refused (no CPU fallback)."""
    g = _rand_graph(n=20, m=50)
    sage = nn.SAGEConv(4, 2, "mean")
    with pytest.raises(Exception):
        sage(g, th.randn(20, 4))


# ----------------------------------------------------------------- dense forms
def _random_graph100():
    return dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1, random_state=11), readonly=True)


def _random_bipartite():
    return dgl.bipartite(sp.sparse.random(100, 200, density=0.1, random_state=12))


@pytest.mark.parametrize("norm_type", ["both", "right", "none"])
@pytest.mark.parametrize("kind", ["graph", "bipartite"])
def test_dense_graph_conv(norm_type, kind):
    """test_nn.py:595-610: DenseGraphConv on adjacency_matrix().to_dense() ==
    GraphConv on the graph (same weights)."""
    g = _random_graph100() if kind == "graph" else _random_bipartite()
    adj = g.adjacency_matrix(ctx=DEV).to_dense()
    conv = nn.GraphConv(5, 2, norm=norm_type, bias=True).to(DEV)
    dense = nn.DenseGraphConv(5, 2, norm=norm_type, bias=True).to(DEV)
    dense.weight.data = conv.weight.data
    dense.bias.data = conv.bias.data
    feat = th.randn(g.number_of_src_nodes(), 5, device=DEV)
    assert th.allclose(conv(g, feat), dense(adj, feat), **TOL)


@pytest.mark.parametrize("kind", ["graph", "bipartite"])
def test_dense_sage_conv(kind):
    """test_nn.py:612-632: DenseSAGEConv == SAGEConv 'gcn'."""
    g = _random_graph100() if kind == "graph" else _random_bipartite()
    adj = g.adjacency_matrix(ctx=DEV).to_dense()
    sage = nn.SAGEConv(5, 2, "gcn").to(DEV)
    dense = nn.DenseSAGEConv(5, 2).to(DEV)
    dense.fc.weight.data = sage.fc_neigh.weight.data
    dense.fc.bias.data = sage.fc_neigh.bias.data
    if kind == "bipartite":
        feat = (th.randn(100, 5, device=DEV), th.randn(200, 5, device=DEV))
    else:
        feat = th.randn(100, 5, device=DEV)
    assert th.allclose(sage(g, feat), dense(adj, feat), **TOL)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_dense_cheb_conv(k):
    """test_nn.py:649-665: DenseChebConv == ChebConv at lambda_max = 2; and the
    default lambda (eigvals) against dgl.laplacian_lambda_max."""
    g = _random_graph100()
    adj = g.adjacency_matrix(ctx=DEV).to_dense()
    cheb = nn.ChebConv(5, 2, k).to(DEV)
    dense = nn.DenseChebConv(5, 2, k).to(DEV)
    for i in range(len(cheb.fc)):
        dense.W.data[i] = cheb.fc[i].weight.data.t()
    dense.bias.data = cheb.bias.data
    feat = th.randn(100, 5, device=DEV)
    assert th.allclose(cheb(g, feat, [2.0]), dense(adj, feat, 2.0), **TOL)
    # a symmetric graph: the dense eigen-solver and the host Lanczos agree
    gs = _rand_graph(n=60, m=300, seed=13)
    s, d = _edges(gs)
    sym = dgl.DGLGraph()
    sym.add_nodes(60)
    sym.add_edges(th.cat([s, d]).numpy(), th.cat([d, s]).numpy())
    adj = sym.adjacency_matrix(ctx=DEV).to_dense()
    lam = dgl.laplacian_lambda_max(sym)[0]
    assert th.allclose(cheb(sym, feat[:60]), dense(adj, feat[:60]), rtol=1e-3, atol=1e-3), lam
