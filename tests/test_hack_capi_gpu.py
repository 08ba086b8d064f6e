"""C entries of the hack's extra PackedFuncs (``DGLMIRgcnLayer0/1[Backward]``,
``DGLMINbAccess``; reference ``src/kernel/binary_reduce.cc:398-450``, kernels
``src/kernel/cuda/binary_reduce_impl.cu:779-1250``) called through the C ABI,
against fp64 restatements of the reference kernels' sums and against the Python
path (``dgl.backend.rgcn_layer0/1``).  Where the hack's kernels are wrong (the
layer-0 backward overwrites repeated (source, relation) pairs, :1004) the C
entries return the exact sums; the restatements here are the exact sums."""
import numpy as np
import pytest
import torch as th

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(n, m, R, seed, hub=False):
    import dgl
    from graphs import powerlaw
    rng = np.random.default_rng(seed)
    if hub:
        src, dst, n = powerlaw(n, m, seed=seed)
    else:
        src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    # repeated (source, relation) pairs on purpose: the hack's layer-0 backward loses them
    src[: m // 10] = src[0]
    et = rng.integers(0, R, m)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(DEV)
    norm = th.from_numpy(rng.uniform(0.1, 1.0, (m, 1))).float().to(DEV)
    return g, gidx, th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV), \
        th.from_numpy(et).to(DEV), norm


@pytest.mark.parametrize("F,hub", [(16, False), (7, False), (64, True)])
def test_rgcn_layer0_fwd_bwd(F, hub):
    from dgl import kernel as K
    n, m, R = 600, 8000, 3
    g, gidx, s, d, et, norm = _graph(n, m, R, seed=F, hub=hub)
    n = g.number_of_nodes()
    w = th.randn(R, n, F, device=DEV)
    ret = th.full((n, F), float("nan"), device=DEV)
    K.rgcn_layer0(gidx, w, norm, ret, etypes=et.int())
    ref = th.zeros(n, F, dtype=th.float64, device=DEV).index_add_(
        0, d, w.double()[et, s] * norm.double())
    mass = th.zeros(n, F, dtype=th.float64, device=DEV).index_add_(
        0, d, (w.double()[et, s] * norm.double()).abs())
    assert ((ret.double() - ref).abs() <= 1e-5 + 1e-6 * mass).all()
    go = th.randn(n, F, device=DEV)
    gw = th.full((R, n, F), float("nan"), device=DEV)
    K.rgcn_layer0_backward(gidx, go, norm, gw, etypes=et.int())
    gref = th.zeros(R * n, F, dtype=th.float64, device=DEV).index_add_(
        0, et * n + s, go.double()[d] * norm.double()).view(R, n, F)
    th.testing.assert_close(gw.double(), gref, rtol=1e-5, atol=1e-5)
    # same as the Python path's autograd (typed gather)
    from dgl import backend as B
    g.edata["t"] = et
    wr = w.clone().requires_grad_()
    out = B.rgcn_layer0(g, wr, norm, et)
    out.backward(go)
    th.testing.assert_close(out.detach(), ret, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(wr.grad, gw, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("K_in,X,hub", [(16, 16, False), (32, 8, True), (20, 5, False)])
def test_rgcn_layer1_fwd_bwd(K_in, X, hub):
    _layer1_fwd_bwd(K_in, X, hub, 700, 9000)


@pytest.mark.parametrize("K_in,X", [(64, 64), (20, 5), (128, 32)])
def test_rgcn_layer1_tall_gemms(K_in, X):
    """Node counts >= 4096 take the tall-skinny MFMA products (k_gemm_rows with B in
    LDS for X . W and gY . W^T, k_gemm_tn for the row reduction X^T . gY), incl.
    partial row tiles and widths that are not multiples of 32."""
    _layer1_fwd_bwd(K_in, X, False, 40001, 200000)


@pytest.mark.parametrize("X,R,hub,cached_norm,tile", [
    (64, 4, False, True, "16"), (64, 4, True, False, "16"), (32, 2, False, True, "16"),
    (100, 2, True, True, "16"), (64, 4, True, True, "16"), (64, 4, True, True, "32"),
    (100, 2, False, False, "32")])
def test_rgcn_layer1_fused(X, R, hub, cached_norm, tile, monkeypatch):
    """The fused layer-1 kernels (prepared state bit 2: relation-major CSRs; each
    relation's rows aggregated into LDS, then one MFMA pass by W_t -- no Y = X W_cat
    table): forward and both gradients vs the fp64 restatement and the Python path,
    with the norm streamed from the state or gathered by edge id, on 16-row tiles
    (k_rgcn_fused16, the default) and 32-row tiles (DGLMI_RGCN_TILE=32)."""
    monkeypatch.setenv("DGLMI_RGCN_TILE", tile)
    _layer1_fwd_bwd(64, X, hub, 40001, 200000, R=R, prepare=4, cached_norm=cached_norm)


def _layer1_fwd_bwd(K_in, X, hub, n, m, R=4, prepare=0, cached_norm=True):
    from dgl import kernel as K
    g, gidx, s, d, et, norm = _graph(n, m, R, seed=K_in + X, hub=hub)
    n = g.number_of_nodes()
    gidx.__dict__.pop("_rgcn_state", None)
    et32 = et.int()
    if prepare:
        K.rgcn_prepare(gidx, norm if cached_norm else None, R, layers=prepare, etypes=et32)
        assert gidx._rgcn_state.matches(et32, R, 1)
    h = th.randn(n, K_in, device=DEV)
    w = th.randn(R, K_in, X, device=DEV) / 4
    ret = th.full((n, X), float("nan"), device=DEV)
    K.rgcn_layer1(gidx, h, w, norm, ret, etypes=et32)
    msg = th.einsum("ek,ekx->ex", h.double()[s], w.double()[et]) * norm.double()
    ref = th.zeros(n, X, dtype=th.float64, device=DEV).index_add_(0, d, msg)
    mass = th.zeros(n, X, dtype=th.float64, device=DEV).index_add_(0, d, msg.abs())
    assert ((ret.double() - ref).abs() <= 1e-4 + 1e-5 * mass).all()
    go = th.randn(n, X, device=DEV)
    gh = th.full((n, K_in), float("nan"), device=DEV)
    gw = th.full((R, K_in, X), float("nan"), device=DEV)
    K.rgcn_layer1_backward(gidx, h, w, norm, go, gh, gw, etypes=et32)
    gidx.__dict__.pop("_rgcn_state", None)
    gmsg = go.double()[d] * norm.double()                        # (E, X)
    gh_ref = th.zeros(n, K_in, dtype=th.float64, device=DEV).index_add_(
        0, s, th.einsum("ex,ekx->ek", gmsg, w.double()[et]))
    gw_ref = th.zeros(R, K_in, X, dtype=th.float64, device=DEV).index_add_(
        0, et, th.einsum("ek,ex->ekx", h.double()[s], gmsg))
    # a hub source's gradient sums thousands of out-edge terms: the bound scales with
    # their absolute mass, like the forward's (a flat rtol = 1e-4 failed one hub entry at
    # 1.7e-4 relative, 8.8e-4 absolute, on 16-row tiles)
    gh_mass = th.zeros(n, K_in, dtype=th.float64, device=DEV).index_add_(
        0, s, th.einsum("ex,ekx->ek", gmsg.abs(), w.double()[et].abs()))
    assert ((gh.double() - gh_ref).abs() <= 1e-4 + 1e-5 * gh_mass).all(), \
        float(((gh.double() - gh_ref).abs() / (1e-4 + 1e-5 * gh_mass)).max())
    # the weight gradient sums tens of thousands of terms per entry: the bound scales
    # with their absolute mass, as for the other long fp32 sums
    gw_mass = th.zeros(R, K_in, X, dtype=th.float64, device=DEV).index_add_(
        0, et, th.einsum("ek,ex->ekx", h.double()[s].abs(), gmsg.abs()))
    assert ((gw.double() - gw_ref).abs() <= 2e-4 + 1e-6 * gw_mass).all(), \
        float(((gw.double() - gw_ref).abs() / (2e-4 + 1e-6 * gw_mass)).max())
    # the Python path (GEMM + typed gather, autograd) agrees
    from dgl import backend as B
    hr, wr = h.clone().requires_grad_(), w.clone().requires_grad_()
    out = B.rgcn_layer1(g, hr, wr, norm, et)
    out.backward(go)
    # (two fp32 summation orders, e.g. the fused path's aggregate-then-transform:
    # bounds scaled by the absolute mass of the sums, as against fp64 above)
    assert ((out.detach().double() - ret.double()).abs() <= 2e-4 + 2e-5 * mass).all()
    assert ((hr.grad.double() - gh.double()).abs() <= 2e-4 + 2e-5 * gh_mass).all()
    assert ((wr.grad.double() - gw.double()).abs() <= 4e-4 + 2e-6 * gw_mass).all()


def test_rgcn_gemm_split_k_large_n():
    """Layer-1 weight gradient over many nodes takes the split-K GEMM path."""
    from dgl import kernel as K
    n, m, R, K_in, X = 60000, 200000, 2, 8, 8
    g, gidx, s, d, et, norm = _graph(n, m, R, seed=3)
    h = th.randn(n, K_in, device=DEV)
    w = th.randn(R, K_in, X, device=DEV)
    go = th.randn(n, X, device=DEV)
    gh = th.empty(n, K_in, device=DEV)
    gw = th.empty(R, K_in, X, device=DEV)
    K.rgcn_layer1_backward(gidx, h, w, norm, go, gh, gw, etypes=et.int())
    gmsg = go.double()[d] * norm.double()
    gw_ref = th.zeros(R, K_in, X, dtype=th.float64, device=DEV).index_add_(
        0, et, th.einsum("ek,ex->ekx", h.double()[s], gmsg))
    th.testing.assert_close(gw.double(), gw_ref, rtol=1e-4, atol=1e-3)


def test_rgcn_rejects_bad_arguments():
    from dgl import kernel as K
    from dgl._ffi import DGLError
    g, gidx, s, d, et, norm = _graph(100, 500, 2, seed=1)
    w = th.randn(2, 100, 8, device=DEV)
    ret = th.empty(100, 8, device=DEV)
    with pytest.raises(DGLError, match="etypes"):
        K.rgcn_layer0(gidx, w, norm, ret, etypes=et[:10].int())
    with pytest.raises(DGLError, match="norm"):
        K.rgcn_layer0(gidx, w, norm[:10], ret, etypes=et.int())
    with pytest.raises(DGLError, match="source nodes"):
        K.rgcn_layer0(gidx, th.randn(2, 50, 8, device=DEV), norm, ret, etypes=et.int())
    with pytest.raises(DGLError, match="edge types"):  # an untyped graph, no etypes given
        K.rgcn_layer0(gidx, w, norm, ret)


def test_nb_access_times_the_gather():
    from dgl import backend as B
    g, gidx, s, d, et, norm = _graph(5000, 60000, 2, seed=2)
    x = th.randn(5000, 64, device=DEV)
    out, us = B.nb_access_bench(g, x, None, None, times=6, warm_up_times=2)
    assert out is x and us > 0


def _layer_calls(K, gidx, et32, norm, n, R, layer, seed):
    """forward + backward of one hack layer through the C entries (fixed inputs)."""
    gen = th.Generator(device=DEV).manual_seed(seed)
    if layer == 0:
        F = 16
        w = th.randn(R, n, F, device=DEV, generator=gen)
        go = th.randn(n, F, device=DEV, generator=gen)
        ret = th.empty(n, F, device=DEV)
        gw = th.empty(R, n, F, device=DEV)
        K.rgcn_layer0(gidx, w, norm, ret, etypes=et32)
        K.rgcn_layer0_backward(gidx, go, norm, gw, etypes=et32)
        return ret, gw
    K_in, X = 32, 16
    h = th.randn(n, K_in, device=DEV, generator=gen)
    w = th.randn(R, K_in, X, device=DEV, generator=gen) / 4
    go = th.randn(n, X, device=DEV, generator=gen)
    ret = th.empty(n, X, device=DEV)
    gh, gw = th.empty(n, K_in, device=DEV), th.empty(R, K_in, X, device=DEV)
    K.rgcn_layer1(gidx, h, w, norm, ret, etypes=et32)
    K.rgcn_layer1_backward(gidx, h, w, norm, go, gh, gw, etypes=et32)
    return ret, gh, gw


@pytest.mark.parametrize("layer", [0, 1])
def test_rgcn_prepared_state_bit_identical(layer):
    """DGLMIRgcnPrepare (relation-expanded columns, typed out-CSR and norm in
    position order built once per graph): every entry returns the same bits as the
    stateless call; a different norm tensor, or an in-place write into the cached one,
    re-gathers the cached copies (DGLMIRgcnRefreshNorm) and keeps the same bits."""
    from dgl import kernel as K
    g, gidx, s, d, et, norm = _graph(700, 9000, 4, seed=21 + layer, hub=True)
    n, R = g.number_of_nodes(), 4
    et32 = et.int()
    gidx.__dict__.pop("_rgcn_state", None)
    plain = _layer_calls(K, gidx, et32, norm, n, R, layer, seed=5)
    st = K.rgcn_prepare(gidx, norm, R, layers=1 << layer, etypes=et32)
    assert st.c.owner and st.c.nnz == len(s)
    prepared = _layer_calls(K, gidx, et32, norm, n, R, layer, seed=5)
    for a, b in zip(plain, prepared):
        assert th.equal(a, b)
    norm2 = norm * 2 + 0.5
    gidx.__dict__.pop("_rgcn_state")
    plain2 = _layer_calls(K, gidx, et32, norm2, n, R, layer, seed=6)
    gidx.__dict__["_rgcn_state"] = st
    for a, b in zip(plain2, _layer_calls(K, gidx, et32, norm2, n, R, layer, seed=6)):
        assert th.equal(a, b)
    assert st.norm is norm2  # re-gathered, not rebuilt
    norm2.mul_(3.0)  # in place: the cached copy is stale and must be re-gathered
    gidx.__dict__.pop("_rgcn_state")
    plain3 = _layer_calls(K, gidx, et32, norm2, n, R, layer, seed=7)
    gidx.__dict__["_rgcn_state"] = st
    assert st.matches(et32, R, layer)
    for a, b in zip(plain3, _layer_calls(K, gidx, et32, norm2, n, R, layer, seed=7)):
        assert th.equal(a, b)
    assert st.versions[1] == norm2._version
    # other relation ids (another tensor) do not match the state
    assert not st.matches(et32.clone(), R, layer)
    gidx.__dict__.pop("_rgcn_state")


def test_rgcn_prepare_rejects_bad_arguments():
    from dgl import kernel as K
    from dgl._ffi import DGLError
    g, gidx, s, d, et, norm = _graph(100, 500, 2, seed=1)
    with pytest.raises(DGLError, match="layers"):
        K.RgcnState(gidx, norm, 2, 8, etypes=et.int())
    with pytest.raises(DGLError, match="norm"):
        K.RgcnState(gidx, norm[:10], 2, 3, etypes=et.int())
    with pytest.raises(DGLError, match="etypes"):
        K.RgcnState(gidx, norm, 2, 3, etypes=et.int()[:10])


@pytest.mark.parametrize("K_in,X,R,prepare,hub,tile", [
    (64, 64, 4, 6, True, "16"), (64, 32, 3, 6, False, "16"), (64, 64, 4, 0, False, "16"),
    (24, 16, 2, 2, True, "16"), (64, 64, 4, 6, True, "32"), (64, 100, 2, 6, False, "16")])
def test_rgcn_layer1_ex_self_loop(K_in, X, R, prepare, hub, tile, monkeypatch):
    """DGLMIRgcnLayer1Ex / BackwardEx: the relation sum + hidden . loop_weight + bias
    (+ addend) forward, and grad_hidden with the self-loop term plus grad_loop_weight,
    vs fp64 -- on the fused kernels (64-wide rows, prepared state: the self-loop is one
    more MFMA pass over the tile's own rows; 16- and 32-row tiles) and on the GEMM +
    gather path."""
    from dgl import kernel as K
    monkeypatch.setenv("DGLMI_RGCN_TILE", tile)
    g, gidx, s, d, et, norm = _graph(20001, 150000, R, seed=K_in + X + R, hub=hub)
    n = g.number_of_nodes()
    gidx.__dict__.pop("_rgcn_state", None)
    et32 = et.int()
    if prepare:
        K.rgcn_prepare(gidx, norm, R, layers=prepare, etypes=et32)
    h = th.randn(n, K_in, device=DEV)
    w = th.randn(R, K_in, X, device=DEV) / 4
    lw = th.randn(K_in, X, device=DEV) / 4
    bias = th.randn(X, device=DEV)
    add = th.randn(n, X, device=DEV)
    msg = th.einsum("ek,ekx->ex", h.double()[s], w.double()[et]) * norm.double()
    agg = th.zeros(n, X, dtype=th.float64, device=DEV).index_add_(0, d, msg)
    mass = th.zeros(n, X, dtype=th.float64, device=DEV).index_add_(0, d, msg.abs())
    loop = h.double() @ lw.double()
    lmass = h.double().abs() @ lw.double().abs()
    for addend in (None, add):
        ret = th.full((n, X), float("nan"), device=DEV)
        K.rgcn_layer1_ex(gidx, h, w, norm, ret, loop_weight=lw, bias=bias, addend=addend,
                         etypes=et32)
        ref = agg + bias.double() + loop + (0 if addend is None else addend.double())
        assert ((ret.double() - ref).abs() <= 1e-4 + 1e-5 * (mass + lmass)).all()
    go = th.randn(n, X, device=DEV)
    gh = th.full((n, K_in), float("nan"), device=DEV)
    gw = th.full((R, K_in, X), float("nan"), device=DEV)
    gl = th.full((K_in, X), float("nan"), device=DEV)
    K.rgcn_layer1_backward_ex(gidx, h, w, norm, lw, go, gh, gw, gl, etypes=et32)
    gmsg = go.double()[d] * norm.double()
    gh_ref = th.zeros(n, K_in, dtype=th.float64, device=DEV).index_add_(
        0, s, th.einsum("ex,ekx->ek", gmsg, w.double()[et])) + go.double() @ lw.double().t()
    gh_mass = th.zeros(n, K_in, dtype=th.float64, device=DEV).index_add_(
        0, s, th.einsum("ex,ekx->ek", gmsg.abs(), w.double()[et].abs())) + \
        go.double().abs() @ lw.double().abs().t()
    assert ((gh.double() - gh_ref).abs() <= 1e-4 + 1e-5 * gh_mass).all()
    gw_ref = th.zeros(R, K_in, X, dtype=th.float64, device=DEV).index_add_(
        0, et, th.einsum("ek,ex->ekx", h.double()[s], gmsg))
    gw_mass = th.zeros(R, K_in, X, dtype=th.float64, device=DEV).index_add_(
        0, et, th.einsum("ek,ex->ekx", h.double()[s].abs(), gmsg.abs()))
    assert ((gw.double() - gw_ref).abs() <= 2e-4 + 1e-6 * gw_mass).all()
    gl_ref = h.double().t() @ go.double()
    gl_mass = h.double().abs().t() @ go.double().abs()
    assert ((gl.double() - gl_ref).abs() <= 2e-4 + 1e-6 * gl_mass).all()
    # no loop weight: the plain entries' results
    ret0, ret1 = th.empty(n, X, device=DEV), th.empty(n, X, device=DEV)
    K.rgcn_layer1(gidx, h, w, norm, ret0, etypes=et32)
    K.rgcn_layer1_ex(gidx, h, w, norm, ret1, etypes=et32)
    assert th.equal(ret0, ret1)
    gidx.__dict__.pop("_rgcn_state", None)


def test_rgcn_layer1_ex_rejects_bad_arguments():
    from dgl import kernel as K
    from dgl._ffi import DGLError
    g, gidx, s, d, et, norm = _graph(3000, 20000, 2, seed=3)
    n = g.number_of_nodes()
    et32 = et.int()
    h, w = th.randn(n, 16, device=DEV), th.randn(2, 16, 8, device=DEV)
    ret = th.empty(n, 8, device=DEV)
    with pytest.raises(DGLError, match="loop_weight"):
        K.rgcn_layer1_ex(gidx, h, w, norm, ret, loop_weight=th.randn(8, 16, device=DEV),
                         etypes=et32)
    with pytest.raises(DGLError, match="grad_loop_weight needs loop_weight"):
        K.rgcn_layer1_backward_ex(gidx, h, w, norm, None, th.randn(n, 8, device=DEV),
                                  th.empty(n, 16, device=DEV), th.empty_like(w),
                                  th.empty(16, 8, device=DEV), etypes=et32)


@pytest.mark.parametrize("n,m,tile", [(500, 4000, "16"), (1700, 20000, "16"), (33, 300, "16"),
                                      (17, 200, "16"), (500, 4000, "32"), (33, 300, "32")])
def test_rgcn_layer1_fused_small_grids(n, m, tile, monkeypatch):
    """Graphs of few row tiles launch the fused kernels on fewer than eight blocks: the
    tile queues shrink to the grid (every queue has a server); partial last tiles."""
    monkeypatch.setenv("DGLMI_RGCN_TILE", tile)
    _layer1_fwd_bwd(64, 64, False, n, m, R=4, prepare=4)


@pytest.mark.parametrize("prepare", [6, 0])
def test_rgcn_layer1_backward_ex_without_grad_hidden(prepare):
    """BackwardEx with grad_hidden NULL (a first layer over data): the weight and
    self-loop gradients are the ones the full call returns, bit for bit."""
    from dgl import kernel as K
    g, gidx, s, d, et, norm = _graph(20001, 150000, 4, seed=9)
    n = g.number_of_nodes()
    gidx.__dict__.pop("_rgcn_state", None)
    et32 = et.int()
    if prepare:
        K.rgcn_prepare(gidx, norm, 4, layers=prepare, etypes=et32)
    h, w = th.randn(n, 64, device=DEV), th.randn(4, 64, 64, device=DEV) / 4
    lw, go = th.randn(64, 64, device=DEV) / 4, th.randn(n, 64, device=DEV)
    gh, gw, gl = th.empty(n, 64, device=DEV), th.empty_like(w), th.empty_like(lw)
    K.rgcn_layer1_backward_ex(gidx, h, w, norm, lw, go, gh, gw, gl, etypes=et32)
    gw2, gl2 = th.full_like(w, float("nan")), th.full_like(lw, float("nan"))
    K.rgcn_layer1_backward_ex(gidx, h, w, norm, lw, go, None, gw2, gl2, etypes=et32)
    assert th.equal(gw, gw2) and th.equal(gl, gl2)
    gidx.__dict__.pop("_rgcn_state", None)
