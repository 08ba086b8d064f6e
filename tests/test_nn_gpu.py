"""NN-module known answers (tests/pytorch/test_nn.py) on the HIP path."""
import networkx as nx
import numpy as np
import pytest
import torch as th

import dgl
import dgl.nn.pytorch as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _AXWb(A, X, W, b):
    X = th.matmul(X, W)
    Y = th.matmul(A, X.view(X.shape[0], -1)).view_as(X)
    return Y + b


def _adj(g):
    s, d = g.edges()
    n = g.number_of_nodes()
    A = th.zeros(n, n)
    A.index_put_((d, s), th.ones(len(s)), accumulate=True)  # row = dst
    return A.to(DEV)


def test_graph_conv_known_answer():
    """test_nn.py:14-38: GraphConv(norm='none') on path_graph(3) == A X W + b."""
    g = dgl.DGLGraph(nx.path_graph(3))
    adj = _adj(g)
    conv = nn.GraphConv(5, 2, norm="none", bias=True).to(DEV)
    h0 = th.ones(3, 5, device=DEV)
    h1 = conv(g, h0)
    assert len(g.ndata) == 0 and len(g.edata) == 0
    assert th.allclose(h1, _AXWb(adj, h0, conv.weight, conv.bias), rtol=1e-4, atol=1e-4)
    h0 = th.ones(3, 5, 5, device=DEV)
    h1 = conv(g, h0)
    assert th.allclose(h1, _AXWb(adj, h0, conv.weight, conv.bias), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("norm", ["both", "right", "none"])
@pytest.mark.parametrize("fin,fout", [(32, 16), (16, 32)])
def test_graph_conv_dense(norm, fin, fout):
    """GraphConv vs a dense float64 restatement, forward and parameter grads."""
    rng = np.random.default_rng(0)
    n = 300
    src = rng.integers(0, n, 3000)
    dst = rng.integers(0, n, 3000)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    conv = nn.GraphConv(fin, fout, norm=norm).to(DEV)
    x = th.randn(n, fin, device=DEV)
    y = conv(g, x)
    y.sum().backward()
    A = _adj(g).double()
    W, b = conv.weight.detach().double().requires_grad_(), conv.bias.detach().double().requires_grad_()
    xd = x.double()
    dout = th.from_numpy(g.out_degrees().numpy()).to(DEV).double().clamp(min=1)
    din = th.from_numpy(g.in_degrees().numpy()).to(DEV).double().clamp(min=1)
    h = xd * dout.pow(-0.5)[:, None] if norm == "both" else xd
    r = A @ (h @ W)
    if norm == "both":
        r = r * din.pow(-0.5)[:, None]
    elif norm == "right":
        r = r / din[:, None]
    r = r + b
    r.sum().backward()
    assert th.allclose(y.double(), r, rtol=1e-4, atol=1e-4)
    assert th.allclose(conv.weight.grad.double(), W.grad, rtol=1e-3, atol=1e-3)


def uniform_attention(g, shape):
    a = th.ones(shape)
    target_shape = (g.number_of_edges(),) + (1,) * (len(shape) - 1)
    return a / g.in_degrees(g.edges()[1]).view(target_shape).float()


def test_edge_softmax():
    """test_nn.py:269-333."""
    g = dgl.DGLGraph(nx.path_graph(3))
    a = nn.edge_softmax(g, th.ones(g.number_of_edges(), 1, device=DEV))
    assert th.allclose(a.cpu(), uniform_attention(g, a.shape))
    a = nn.edge_softmax(g, th.ones(g.number_of_edges(), 3, 1, device=DEV))
    assert th.allclose(a.cpu(), uniform_attention(g, a.shape))
    g = dgl.DGLGraph()
    g.add_nodes(30)
    for i in range(30):
        for j in range(30):
            g.add_edge(i, j)
    score = th.randn(900, 1, device=DEV).requires_grad_()
    grad = th.randn(900, 1, device=DEV)
    y = th.softmax(score.view(30, 30), dim=0).view(-1, 1)
    y.backward(grad)
    grad_score = score.grad.clone()
    score.grad.zero_()
    y_dgl = nn.edge_softmax(g, score)
    assert len(g.ndata) == 0 and len(g.edata) == 0
    assert th.allclose(y_dgl, y, rtol=1e-4, atol=1e-4)
    y_dgl.backward(grad)
    assert th.allclose(score.grad, grad_score, rtol=1e-4, atol=1e-4)


def test_partial_edge_softmax():
    """test_nn.py:334-362: softmax over a subset of edges."""
    g = dgl.DGLGraph()
    g.add_nodes(30)
    for i in range(30):
        for j in range(30):
            g.add_edge(i, j)
    score = th.randn(300, 1, device=DEV).requires_grad_()
    grad = th.randn(300, 1, device=DEV)
    eids = np.random.permutation(900)[:300]
    eids_t = th.from_numpy(eids)
    s, d = g.edges()
    s, d = s[eids_t], d[eids_t]
    # reference: softmax grouped by destination
    y = th.zeros_like(score)
    for v in range(30):
        m = (d == v).nonzero().view(-1).to(DEV)
        if len(m):
            y = y.index_put((m,), th.softmax(score[m], dim=0))
    y.backward(grad)
    g1 = score.grad.clone()
    score.grad.zero_()
    y_dgl = nn.edge_softmax(g, score, eids_t)
    assert th.allclose(y_dgl, y, rtol=1e-4, atol=1e-4)
    y_dgl.backward(grad)
    assert th.allclose(score.grad, g1, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("use_fused", [False, True])
def test_gat_conv_vs_dense(use_fused):
    """GATConv against a dense torch restatement (float64)."""
    th.manual_seed(0)
    n, fin, H, D = 200, 24, 4, 8
    rng = np.random.default_rng(1)
    src = np.concatenate([rng.integers(0, n, 2000), np.arange(n)])
    dst = np.concatenate([rng.integers(0, n, 2000), np.arange(n)])
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gat = nn.GATConv(fin, D, H).to(DEV)
    gat.use_fused = use_fused
    x = th.randn(n, fin, device=DEV)
    out = gat(g, x)
    assert out.shape == (n, H, D)
    out.sum().backward()
    Wd = gat.fc.weight.detach().double().requires_grad_()
    al = gat.attn_l.detach().double().requires_grad_()
    ar = gat.attn_r.detach().double().requires_grad_()
    ft = (x.double() @ Wd.t()).view(n, H, D)
    el = (ft * al).sum(-1)
    er = (ft * ar).sum(-1)
    s = th.from_numpy(src).to(DEV)
    d = th.from_numpy(dst).to(DEV)
    e = th.nn.functional.leaky_relu(el[s] + er[d], 0.2)  # (E, H)
    emax = th.full((n, H), -1e300, dtype=th.float64, device=DEV).index_reduce(0, d, e, "amax")
    ex = th.exp(e - emax[d])
    den = th.zeros(n, H, dtype=th.float64, device=DEV).index_add(0, d, ex)
    a = ex / den[d]
    rst = th.zeros(n, H, D, dtype=th.float64, device=DEV).index_add(0, d, ft[s] * a[:, :, None])
    rst.sum().backward()
    assert th.allclose(out.double(), rst, rtol=1e-4, atol=1e-4)
    assert th.allclose(gat.fc.weight.grad.double(), Wd.grad, rtol=1e-3, atol=1e-3)
    assert th.allclose(gat.attn_l.grad.double(), al.grad, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("m,k,n", [(5000, 602, 64), (169343, 128, 128), (300001, 64, 32)])
def test_project_split_k_weight_grad(m, k, n):
    """dgl.backend.project: Y = X W with the split-K weight gradient (bmm over node
    slices + sum) equals X^T dY in fp64 to fp32 accuracy; dX = dY W^T."""
    from dgl import backend as B
    g = th.Generator(device=DEV).manual_seed(0)
    x = th.randn(m, k, device=DEV, generator=g).requires_grad_()
    w = th.randn(k, n, device=DEV, generator=g).requires_grad_()
    gy = th.randn(m, n, device=DEV, generator=g)
    y = B.project(x, w)
    y.backward(gy)
    ref_w = x.detach().double().t() @ gy.double()
    ref_x = gy.double() @ w.detach().double().t()
    scale_w = (x.detach().double().abs().t() @ gy.double().abs())
    assert th.allclose(y.double(), x.detach().double() @ w.detach().double(), rtol=1e-4, atol=1e-3)
    assert bool(((w.grad.double() - ref_w).abs() <= 1e-5 * scale_w + 1e-4).all())
    assert th.allclose(x.grad.double(), ref_x, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("k,n", [(16, 64), (32, 128), (64, 64), (64, 128), (128, 128)])
@pytest.mark.parametrize("wt", [False, True])
def test_project_mfma_kernel(k, n, wt):
    """DGLMIProject (the tall-skinny MFMA projection) against fp64: a plain and a
    transposed weight view (nn.Linear's weight.t()), with and without bias, a row count
    that is not a multiple of the 16-row tile; and B.project's forward / dX take it."""
    from dgl import backend as B
    from dgl import kernel as K
    g = th.Generator(device=DEV).manual_seed(k + n)
    m = K.PROJECT_MIN_ROWS + 37
    x = th.randn(m, k, device=DEV, generator=g)
    w = th.randn(n, k, device=DEV, generator=g).t() if wt else th.randn(k, n, device=DEV, generator=g)
    b = th.randn(n, device=DEV, generator=g)
    assert K.project_mfma_ok(x, w)
    ref = x.double() @ w.double()
    mag = x.double().abs() @ w.double().abs()
    for bias in (None, b):
        y = K.project_mfma(x, w, bias)
        r = ref if bias is None else ref + bias.double()
        assert bool(((y.double() - r).abs() <= 2e-6 * mag + 1e-6).all())
    xr = x.clone().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    gy = th.randn(m, n, device=DEV, generator=g)
    B.project(xr, wr).backward(gy)
    gref = gy.double() @ wr.detach().double().t()
    gmag = gy.double().abs() @ wr.detach().double().abs().t()
    assert bool(((xr.grad.double() - gref).abs() <= 2e-6 * gmag + 1e-6).all())


@pytest.mark.parametrize("k,n", [(602, 64), (64, 602), (64, 256), (256, 64), (100, 128), (3, 7),
                                 (17, 41), (300, 33), (640, 50), (64, 1000), (32, 256), (16, 200),
                                 (200, 100), (500, 64), (250, 64), (63, 200), (601, 64)])
@pytest.mark.parametrize("wt", [False, True])
def test_project_tile_kernel(k, n, wt):
    """k_project_tile (X tiles staged through LDS, waves split over columns or k): any
    K <= 640 (GATConv's 602 -> 64 on Reddit and its dX 64 -> 602), wide N (R-GCN's
    64 -> 256 with one X read), odd widths (per-element LDS staging of a row span that is
    not float4-aligned; float2 / scalar stores), a row count off the 16-row tile, plain
    and transposed weights, with and without bias -- against fp64 (every instance of
    kernels_project.hip's table: 16 / 32 / 64 x 256, 64 x 640, 128 x 128, 256 x 128,
    256 / 512 / 640 x 64; each in its K % 4 == 0, K even and K odd LDS image)."""
    from dgl import kernel as K
    g = th.Generator(device=DEV).manual_seed(3 * k + n)
    m = K.PROJECT_MIN_ROWS + 21
    x = th.randn(m, k, device=DEV, generator=g)
    w = th.randn(n, k, device=DEV, generator=g).t() if wt else th.randn(k, n, device=DEV, generator=g)
    b = th.randn(n, device=DEV, generator=g)
    assert K.project_mfma_ok(x, w)
    ref = x.double() @ w.double()
    mag = x.double().abs() @ w.double().abs()
    for bias in (None, b):
        y = K.project_mfma(x, w, bias)
        r = ref if bias is None else ref + bias.double()
        err = (y.double() - r).abs() - (2e-6 * mag + 1e-6)
        assert bool((err <= 0).all()), float(err.max())


def test_project_k_mismatch_raises():
    """An (M, 128) X against a (64, 64) W: torch.matmul raises, so B.project does, and
    the C entry -- handed the weight's row count -- refuses it (DGLError) instead of
    reading W rows 64..127 out of bounds."""
    from dgl import backend as B
    from dgl import kernel as K
    from dgl._ffi import DGLError
    x = th.randn(K.PROJECT_MIN_ROWS, 128, device=DEV)
    w = th.randn(64, 64, device=DEV)
    assert not K.project_mfma_ok(x, w)
    with pytest.raises(RuntimeError):
        B.project(x, w)
    with pytest.raises(DGLError, match="rows"):
        K.project_mfma(x, w)


def test_project_misaligned_bias_slice():
    """A bias that is a slice of a flat parameter buffer at an offset of 1 float (not
    16-byte aligned) takes torch.addmm instead of raising, and matches fp64."""
    from dgl import backend as B
    from dgl import kernel as K
    g = th.Generator(device=DEV).manual_seed(9)
    m = K.PROJECT_MIN_ROWS + 5
    x = th.randn(m, 64, device=DEV, generator=g)
    w = th.randn(64, 64, device=DEV, generator=g)
    flat = th.randn(65, device=DEV, generator=g)
    bias = flat[1:]
    assert bias.data_ptr() % 16 != 0 and not K.project_bias_ok(bias, 64, x.device)
    y = B.project(x, w, bias)
    ref = x.double() @ w.double() + bias.double()
    mag = x.double().abs() @ w.double().abs()
    assert bool(((y.double() - ref).abs() <= 2e-6 * mag + 1e-5).all())
    # an aligned slice of the same buffer rides in the kernel's epilogue
    flat4 = th.randn(68, device=DEV, generator=g)
    b4 = flat4[4:]
    assert K.project_bias_ok(b4, 64, x.device)
    y4 = B.project(x, w, b4)
    ref4 = x.double() @ w.double() + b4.double()
    assert bool(((y4.double() - ref4).abs() <= 2e-6 * mag + 1e-5).all())


def test_nb_access_bench():
    """The hack's neighbour-access benchmark entry point returns feat and a time."""
    from dgl import backend as B
    g = dgl.DGLGraph()
    g.add_nodes(100)
    g.add_edges(np.arange(100), (np.arange(100) + 1) % 100)
    x = th.randn(100, 16, device=DEV)
    y, us = B.nb_access_bench(g, x, None, None)
    assert y is x and us > 0


@pytest.mark.parametrize("shape", [(), (2,), (4, 1), (8, 1), (16,), (3, 1)],
                         ids=["1", "2", "4x1", "8x1", "16", "3x1-decomposed"])
def test_fused_edge_softmax_vs_decomposition(shape):
    """kernels_softmax.hip (online max / sum per destination, chunk-merged on hub
    rows) against the reference's five-kernel decomposition and an fp64 softmax
    per destination, forward and backward, on a power-law graph."""
    from dgl.nn.pytorch import softmax as S
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 60000, seed=9)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    m = len(src)
    rs = np.random.RandomState(2)
    s = th.from_numpy((rs.randn(m, *shape) * 3).astype(np.float32)).to(DEV)
    go = th.from_numpy(rs.randn(m, *shape).astype(np.float32)).to(DEV)
    res = {}
    for fused in (True, False):
        S.FUSED = fused
        try:
            x = s.clone().requires_grad_()
            a = nn.edge_softmax(g, x)
            a.backward(go)
            res[fused] = (a.detach(), x.grad)
        finally:
            S.FUSED = True
    (a1, g1), (a0, g0) = res[True], res[False]
    assert th.allclose(a1, a0, rtol=1e-5, atol=1e-6)
    assert th.allclose(g1, g0, rtol=1e-4, atol=1e-5)
    # fp64 softmax per destination
    d = th.from_numpy(dst).to(DEV)
    s64 = s.double().reshape(m, -1)
    mx = th.full((n, s64.shape[1]), -float("inf"), dtype=th.float64, device=DEV)
    mx = mx.index_reduce(0, d, s64, "amax")
    ex = th.exp(s64 - mx[d])
    den = th.zeros_like(mx).index_add_(0, d, ex)
    ref = (ex / den[d]).reshape(a1.shape)
    assert th.allclose(a1.double(), ref, rtol=1e-5, atol=1e-7)


def test_fused_edge_softmax_masked_logits():
    """-inf logits (masked edges) get probability 0; a row of all -inf gives NaN,
    as the decomposition does (exp(-inf - -inf))."""
    from dgl.nn.pytorch import softmax as S
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 1, 2, 0], [1, 1, 1, 2])
    # row 1 sees its in-edges in source order 0, 1, 2: a masked logit first
    x = th.tensor([[-float("inf")], [0.5], [1.5], [-float("inf")]], device=DEV)
    a = nn.edge_softmax(g, x)
    S.FUSED = False
    try:
        b = nn.edge_softmax(g, x)
    finally:
        S.FUSED = True
    assert a[0].item() == 0.0
    assert th.allclose(a[[1, 2]], b[[1, 2]], rtol=1e-6)
    assert bool(th.isnan(a[3]).all()) and bool(th.isnan(b[3]).all())


@pytest.mark.parametrize("norm", ["none", "both", "right"])
@pytest.mark.parametrize("weight", [True, False])
@pytest.mark.parametrize("bias", [True, False])
def test_graph_conv2_external_weight(norm, weight, bias):
    """test_nn.py:72-88: module weight or an external one (weight=False), with or
    without bias, every norm; plus reset_parameters (test_nn.py:66-70)."""
    g = dgl.DGLGraph(nx.path_graph(3))
    conv = nn.GraphConv(5, 2, norm=norm, weight=weight, bias=bias).to(DEV)
    ext_w = th.randn(5, 2, device=DEV)
    h = th.randn(3, 5, device=DEV)
    out = conv(g, h) if weight else conv(g, h, weight=ext_w)
    assert out.shape == (3, 2)
    w = conv.weight if weight else ext_w
    ref = nn.GraphConv(5, 2, norm=norm, weight=False, bias=False).to(DEV)(g, h, weight=w)
    if bias:
        ref = ref + conv.bias
    assert th.allclose(out, ref, rtol=1e-5, atol=1e-6)
    if weight:
        old = conv.weight.detach().clone()
        conv.reset_parameters()
        assert not th.allclose(old, conv.weight)


def test_rgcn_reference_shapes():
    """test_nn.py:363-407 on a readonly scipy-built graph: basis / bdd, with a
    per-edge norm, and integer id input."""
    import scipy as sp
    import scipy.sparse  # noqa: F401
    g = dgl.DGLGraph(sp.sparse.random(100, 100, density=0.1, random_state=0), readonly=True)
    R, B, I, O = 5, 2, 10, 8
    r = th.tensor([i % 5 for i in range(g.number_of_edges())], device=DEV)
    norm = th.zeros(g.number_of_edges(), 1, device=DEV)
    for reg in ("basis", "bdd"):
        conv = nn.RelGraphConv(I, O, R, reg, B).to(DEV)
        h = th.randn(100, I, device=DEV)
        assert list(conv(g, h, r).shape) == [100, O]
        out = conv(g, h, r, norm)
        assert list(out.shape) == [100, O]
        assert th.allclose(out, conv.h_bias.expand(100, O))  # zero norm: only the bias
    conv = nn.RelGraphConv(I, O, R, "basis", B).to(DEV)
    h = th.randint(0, I, (100,), device=DEV)
    assert list(conv(g, h, r).shape) == [100, O]


@pytest.mark.parametrize("blocks", [None, "2"])
@pytest.mark.parametrize("norm", ["none", "both", "right"])
@pytest.mark.parametrize("fin,fout", [(64, 16), (16, 64), (32, 12), (8, 8)])
def test_graph_conv_fused_epilogue_matches_reference_steps(norm, fin, fout, blocks, monkeypatch):
    """The fused paths against the reference's separate steps: outputs and all
    gradients on a power-law graph with empty rows.  Default: norms 'both' /
    'right' as one streamed weight per edge (gcn_norm_aggregate); with column
    blocks forced (DGLMI_SPMM_BLOCKS=2) the copy_u sum with the norm * sum + bias
    epilogue, chained over the blocks."""
    if blocks is not None:
        monkeypatch.setenv("DGLMI_SPMM_BLOCKS", blocks)
    from graphs import powerlaw
    src, dst, n = powerlaw(4000, 60000, seed=11)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    th.manual_seed(3)
    conv = nn.GraphConv(fin, fout, norm=norm, activation=th.relu).to(DEV)
    with th.no_grad():
        conv.bias.uniform_(-1, 1)
    x = th.randn(n, fin, device=DEV)
    res = []
    for fused in (True, False):
        conv.fused = fused
        conv.zero_grad()
        xi = x.clone().requires_grad_()
        y = conv(g, xi)
        y.backward(th.ones_like(y))
        res.append((y.detach(), xi.grad, conv.weight.grad.clone(), conv.bias.grad.clone()))
    for a, b in zip(*res):
        assert th.allclose(a, b, rtol=1e-4, atol=1e-4)
    if fin > fout and (norm == "none" or blocks is not None):
        # same order of operations as the reference: bit-identical forward
        # (blocks: the first block's partial sums restart the chain, so only
        # the unblocked epilogue path keeps the order)
        if blocks is None:
            assert th.equal(res[0][0], res[1][0])


@pytest.mark.parametrize("owned", ["0", "1"])
@pytest.mark.parametrize("H,D", [(8, 8), (3, 5), (1, 16)])
def test_gat_composition_position_space_bit_identical(H, D, owned, monkeypatch):
    """GATConv's unfused composition run on the in-CSR position view (logits and
    attention in walk order, GATConv._position_space) gives the same bits as the
    edge-id composition: output and every gradient, when the view's edge softmax runs
    the same chunked kernels (DGLMI_SOFTMAX_OWNED=0).  With the row-owned softmax the
    view's (the default since round 5: one read per logit, another summation order) the
    results agree within fp32 tolerance.  (3 heads: the edge softmax's decomposition
    rather than its fused kernel.)"""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
    from dgl.nn.pytorch.conv import gatconv
    from graphs import powerlaw
    monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", False)  # step by step
    src, dst, n = powerlaw(20000, 300000, seed=21)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    th.manual_seed(3)
    gat = nn.GATConv(32, D, H).to(DEV)
    gat.use_fused = False
    x = th.randn(n, 32, device=DEV, requires_grad=True)
    go = th.randn(n, H, D, device=DEV)
    res = []
    for pos in (True, False):
        monkeypatch.setattr(gatconv, "POSITION_SPACE", pos)
        calls = []
        orig = gat._composed_in_positions
        monkeypatch.setattr(gat, "_composed_in_positions", lambda *a: calls.append(1) or orig(*a))
        gat.zero_grad()
        x.grad = None
        out = gat(g, x)
        out.backward(go)
        assert bool(calls) == pos
        res.append([out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in gat.parameters()])
    for a, b in zip(*res):
        if owned == "0" or H == 3:
            assert th.equal(a, b), float((a - b).abs().max())
        else:
            assert th.allclose(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max())), \
                float((a - b).abs().max())
    # attention dropout in training: nn.Dropout's edge-id-order draws gathered into
    # walk order (the same kept edges, the same bits with the same softmax kernels)
    gd = nn.GATConv(32, D, H, attn_drop=0.5).to(DEV)
    gd.use_fused = False
    monkeypatch.setattr(gatconv, "POSITION_SPACE", True)
    assert gd._position_space(g, x) and gd.eval()._position_space(g, x)
    gd.train()
    gd.attn_drop.inplace = True  # a dropout that writes its input keeps the edge-id route
    assert not gd._position_space(g, x)
    gd.attn_drop.inplace = False
    res = []
    for pos in (True, False):
        monkeypatch.setattr(gatconv, "POSITION_SPACE", pos)
        gd.zero_grad()
        x.grad = None
        th.manual_seed(11)
        out = gd(g, x)
        out.backward(go)
        res.append([out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in gd.parameters()])
    assert float((res[0][0] == 0).float().mean()) < 0.9  # dropout did not zero everything
    for a, b in zip(*res):
        if owned == "0" or H == 3:
            assert th.equal(a, b), float((a - b).abs().max())
        else:
            assert th.allclose(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max())), \
                float((a - b).abs().max())


@pytest.mark.parametrize("pos", [True, False])
@pytest.mark.parametrize("owned", ["0", "1"])
def test_gat_composition_fused_leaky_bit_identical(pos, owned, monkeypatch):
    """The composition's leaky_relu -> edge_softmax pair as one fused softmax call
    (gatconv.FUSED_LEAKY, DGLMIEdgeSoftmaxLeaky*) gives the two-step form's bits: output
    and every gradient, on the position view and in edge-id order, with either softmax
    route."""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
    from dgl.nn.pytorch.conv import gatconv
    from graphs import powerlaw
    monkeypatch.setattr(gatconv, "POSITION_SPACE", pos)
    monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", False)  # step by step
    src, dst, n = powerlaw(20000, 300000, seed=22)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    th.manual_seed(4)
    gat = nn.GATConv(32, 8, 8, negative_slope=0.15).to(DEV)
    gat.use_fused = False
    x = th.randn(n, 32, device=DEV, requires_grad=True)
    go = th.randn(n, 8, 8, device=DEV)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(gatconv, "FUSED_LEAKY", fused)
        gat.zero_grad()
        x.grad = None
        out = gat(g, x)
        out.backward(go)
        res.append([out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in gat.parameters()])
    for a, b in zip(*res):
        assert th.equal(a, b), float((a - b).abs().max())


@pytest.mark.parametrize("owned", ["0", "1"])
@pytest.mark.parametrize("H,D,blocks", [(8, 8, "1"), (8, 8, "4"), (1, 16, "1"), (4, 32, "1"),
                                        (16, 4, "2"), (2, 8, "1")])
def test_gat_composition_fused_backward(H, D, blocks, owned, monkeypatch):
    """The position-space composition with its backward fused (backend.GatComposition:
    the softmax's row statistics handed to the fused GAT backward walks) against the
    step-by-step backward: the forward bit for bit (the same kernels), the input and every
    parameter gradient within fp32 rounding -- on a power-law graph with hub rows and
    zero-in-degree rows, both softmax routes (the row-owned walk's hub rows included in
    the exported statistics), unblocked (the edge-position path) and column-blocked (the
    destination- and source-side walks).  The fused route is the one taken."""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", blocks)
    from dgl import backend as B
    from dgl.nn.pytorch.conv import gatconv
    from graphs import powerlaw
    src, dst, n = powerlaw(30000, 400000, seed=23 + H)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    th.manual_seed(5)
    gat = nn.GATConv(24, D, H, negative_slope=0.2).to(DEV)
    gat.use_fused = False
    x = th.randn(n, 24, device=DEV, requires_grad=True)
    go = th.randn(n, H, D, device=DEV)
    calls = []
    orig = B.gat_composition
    monkeypatch.setattr(B, "gat_composition", lambda *a: calls.append(1) or orig(*a))
    res = []
    for fused in (True, False):
        monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", fused)
        gat.zero_grad()
        x.grad = None
        out = gat(g, x)
        out.backward(go)
        res.append([out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in gat.parameters()])
    assert calls == [1]
    assert th.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1:], res[1][1:]):
        tol = 1e-4 * float(b.abs().max()) + 1e-7
        assert float((a - b).abs().max()) <= tol, (float((a - b).abs().max()), tol)


@pytest.mark.parametrize("h,d", [(8, 8), (1, 4), (4, 16), (2, 32), (16, 4), (64, 4), (4, 64), (32, 8)])
@pytest.mark.parametrize("two", [False, True])
def test_attn_logits_kernel(h, d, two):
    """DGLMIGatAttnLogits / Backward (GATConv's el / er, gatconv.py:137-138) against fp64:
    one feature table and two (bipartite, n_src != n_dst, both larger), every head layout
    the kernel takes (D / 4 lanes per head: 1 .. 16; H D / 4 slots per row dividing 256),
    row counts off the grid; the parameter gradients from the per-thread partials."""
    from dgl import backend as B
    from dgl import kernel as K
    g = th.Generator(device=DEV).manual_seed(7 * h + d + two)
    ns = 70001
    nd = 50003 if two else ns
    xs = th.randn(ns, h, d, device=DEV, generator=g).requires_grad_()
    xd = th.randn(nd, h, d, device=DEV, generator=g).requires_grad_() if two else xs
    al = th.randn(1, h, d, device=DEV, generator=g).requires_grad_()
    ar = th.randn(1, h, d, device=DEV, generator=g).requires_grad_()
    assert K.attn_logits_ok(xs, xd, al, ar)
    el, er = B.attn_logits(xs, xd, al, ar)
    assert el.shape == (ns, h, 1) and er.shape == (nd, h, 1)
    rl = (xs.double() * al.double()).sum(-1, keepdim=True)
    rr = (xd.double() * ar.double()).sum(-1, keepdim=True)
    ml = (xs.double().abs() * al.double().abs()).sum(-1, keepdim=True)
    mr = (xd.double().abs() * ar.double().abs()).sum(-1, keepdim=True)
    assert bool(((el.double() - rl).abs() <= 1e-6 * ml + 1e-7).all())
    assert bool(((er.double() - rr).abs() <= 1e-6 * mr + 1e-7).all())
    # torch's own fp32 bits (its pairwise summation order; the LeakyReLU branch of
    # el + er is then the reference composition's)
    with th.no_grad():
        assert th.equal(el, (xs * al).sum(-1, keepdim=True))
        assert th.equal(er, (xd * ar).sum(-1, keepdim=True))
    gl = th.randn(ns, h, 1, device=DEV, generator=g)
    gr = th.randn(nd, h, 1, device=DEV, generator=g)
    ins = [xs, al, ar] + ([xd] if two else [])
    got = th.autograd.grad((el, er), ins, (gl, gr))
    ins64 = [t.detach().double().requires_grad_() for t in ins]
    xs64, al64, ar64 = ins64[:3]
    xd64 = ins64[3] if two else xs64
    ref = th.autograd.grad(((xs64 * al64).sum(-1, keepdim=True), (xd64 * ar64).sum(-1, keepdim=True)),
                           ins64, (gl.double(), gr.double()))
    for a, r, t in zip(got, ref, ins):
        # magnitude bound of each gradient: the same sums over |terms|
        scale = r.abs().amax().item() + 1.0
        tol = 1e-6 * scale * (1.0 if t.dim() == 3 and t.shape[0] > 1 else np.sqrt(ns))
        assert a.shape == t.shape
        assert (a.double() - r).abs().max().item() <= tol


def test_attn_logits_unsupported_and_deterministic():
    """Shapes the kernel does not take stay on torch (head size not a multiple of 4, a
    non-power-of-two D / 4, H D / 4 not dividing 256, D > 64, a strided feature view), and the
    parameter gradients are bit-identical run to run (fixed partial order)."""
    from dgl import backend as B
    from dgl import kernel as K
    for h, d in ((8, 6), (4, 12), (3, 20), (65, 4), (3, 8), (1, 128), (2, 256)):
        x = th.randn(100, h, d, device=DEV)
        a = th.randn(1, h, d, device=DEV)
        assert not K.attn_logits_ok(x, x, a, a)
    x = th.randn(100, 8, 16, device=DEV)[:, :, :8]
    a = th.randn(1, 8, 8, device=DEV)
    assert not K.attn_logits_ok(x, x, a, a)
    x = th.randn(300001, 8, 8, device=DEV).requires_grad_()
    al = th.randn(1, 8, 8, device=DEV).requires_grad_()
    ar = th.randn(1, 8, 8, device=DEV).requires_grad_()
    gl, gr = th.randn(300001, 8, 1, device=DEV), th.randn(300001, 8, 1, device=DEV)
    runs = []
    for _ in range(2):
        el, er = B.attn_logits(x, x, al, ar)
        runs.append((el, er) + th.autograd.grad((el, er), (x, al, ar), (gl, gr)))
    for u, v in zip(*runs):
        assert th.equal(u, v)


@pytest.mark.parametrize("drop", [0.0, 0.6])
def test_gatconv_attn_logits_route(monkeypatch, drop):
    """GATConv's fused route with the device el / er against torch's multiply + sum
    (FUSED_ATTN_LOGITS off): the same output bits, every gradient (x, fc, attn_l, attn_r,
    bias) within fp32 rounding, in training with attention dropout under one seed too."""
    from dgl.nn.pytorch.conv import gatconv
    from graphs import powerlaw
    src, dst, n = powerlaw(20000, 400000, seed=5)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    x = th.randn(n, 48, device=DEV)
    res = []
    for flag in (True, False):
        monkeypatch.setattr(gatconv, "FUSED_ATTN_LOGITS", flag)
        th.manual_seed(0)
        conv = nn.GATConv(48, 8, 8, attn_drop=drop).to(DEV)
        conv.train()
        xr = x.clone().requires_grad_()
        th.manual_seed(1)
        y = conv(g, xr)
        gy = th.randn_like(y)
        grads = th.autograd.grad((y * gy).sum(), [xr] + list(conv.parameters()), allow_unused=True)
        res.append((y,) + tuple(grads))
    assert th.equal(res[0][0], res[1][0])  # el / er are torch's bits: the same forward
    for a, b in zip(*res):
        if a is None:
            assert b is None
            continue
        th.testing.assert_close(a, b, rtol=2e-4, atol=2e-5)
