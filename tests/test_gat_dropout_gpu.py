"""Attention dropout inside the fused GAT kernels.  GATConv in training applies
``nn.Dropout`` to the edge softmax (the reference's ``gatconv.py:154``).  Two fused forms:

* the module's own draws (default): torch's fused dropout draws over (E, H, 1) in edge-id
  order, recomputed inside the walks from the generator state (DGLMIFusedGatDraw*, once
  checked against torch.native_dropout) or drawn by torch and packed to one keep word per
  edge (DGLMIFusedGatKeep*) -- the fused module must agree with the unfused composition
  (the reference's shape) under one seed, and the two routes bit for bit;
* the hashed mask (opt-in, DGLMIFusedGatDropout*): the same Bernoulli(1 - p) per edge and
  head from a hash of a seed and the edge id, rebuilt on the host
  (``dgl.kernel.gat_dropout_keep``) for a dense fp64 restatement that applies it to the
  softmax -- unblocked and column-blocked.

Plus the module routing, FusedGATConv's reference behaviour (attn_drop built, never
applied: fusedGatConv.py:80,152) and p = 1."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
from dgl import kernel as K
from dgl.nn.pytorch import GATConv
from graphs import powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dense_gat_dropout(src, dst, n, ft, el, er, slope, keep, p):
    s, d = th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV)
    H = ft.shape[1]
    e = th.nn.functional.leaky_relu(el[s, :, 0] + er[d, :, 0], slope)
    emax = th.full((n, H), -1e300, dtype=th.float64, device=DEV).index_reduce(0, d, e.detach(), "amax")
    ex = th.exp(e - emax[d])
    den = th.zeros(n, H, dtype=th.float64, device=DEV).index_add(0, d, ex)
    a = ex / den[d] * (th.from_numpy(keep).to(DEV).double() * K.gat_dropout_scale(p))
    return th.zeros(n, H, ft.shape[2], dtype=th.float64, device=DEV).index_add(0, d, ft[s] * a[:, :, None])


@pytest.mark.parametrize("nb,p,H,D", [(1, 0.5, 8, 8), (1, 0.1, 8, 8), (4, 0.6, 8, 8),
                                      (8, 0.3, 8, 8), (1, 0.5, 32, 4), (2, 0.4, 3, 16)])
def test_fused_gat_dropout_vs_dense(nb, p, H, D, monkeypatch):
    """(32 heads: every bit of the staged keep mask in use)"""
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", str(nb))
    src, dst, n = powerlaw(20000, 300000, seed=13)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    if nb > 1:
        ib, ob = g._graph.get_immutable_gidx(th.device(DEV)).col_blocks(nb)
        assert all(c.nnz > 0 for c in ib + ob)
    gen = th.Generator(device=DEV).manual_seed(5)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    er = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    seed = 0x1234_5678_9ABC_DEF0 + nb
    out = B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=seed)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gf = th.autograd.grad(out, (ft, el, er), go)
    keep = K.gat_dropout_keep(seed, np.arange(len(src)), H, p)
    assert abs(keep.mean() - (1 - p)) < 0.01
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat_dropout(src, dst, n, fd, eld, erd, 0.2, keep, p)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4), float((out.double() - ref).abs().max())
    for a, b, name in zip(gf, gr, ("ft", "el", "er")):
        assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), (name, float((a.double() - b).abs().max()))
    # the same seed gives the same mask (bit-identical); another seed another one
    assert th.equal(B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=seed), out)
    assert not th.equal(B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=seed + 1), out)


def test_gatconv_training_dropout_runs_fused(monkeypatch):
    """GATConv(attn_drop=0.6) with the hashed mask in training takes the fused kernels (no
    per-edge attention tensor), reproducibly under torch.manual_seed; eval mode has no
    dropout."""
    src, dst, n = powerlaw(5000, 60000, seed=3)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    conv = GATConv(32, 8, 4, attn_drop=0.6).to(DEV)
    conv.attn_drop_mask = "hashed"
    x = th.randn(n, 32, device=DEV)
    calls = []
    orig = B.fused_gat

    def spy(*a, **k):
        calls.append(k.get("attn_drop", 0.0))
        return orig(*a, **k)
    monkeypatch.setattr(B, "fused_gat", spy)
    conv.train()
    th.manual_seed(7)
    y1 = conv(g, x)
    th.manual_seed(7)
    y2 = conv(g, x)
    y3 = conv(g, x)
    assert calls and all(c == 0.6 for c in calls)
    assert th.equal(y1, y2) and not th.equal(y1, y3)
    y1.sum().backward()
    assert conv.attn_l.grad is not None and th.isfinite(conv.attn_l.grad).all()
    conv.eval()
    calls.clear()
    with th.no_grad():
        e1, e2 = conv(g, x), conv(g, x)
    assert calls == [0.0, 0.0] and th.equal(e1, e2)


def test_dropout_over_32_heads_takes_the_composition():
    """The dropout walks stage 32 keep bits per edge: more heads raise in the C entry,
    and GATConv routes such a layer to the composition (nn.Dropout on edge_softmax)."""
    from dgl._ffi import DGLError
    src, dst, n = powerlaw(3000, 30000, seed=4)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    ft = th.randn(n, 64, 4, device=DEV)
    el, er = th.randn(n, 64, 1, device=DEV), th.randn(n, 64, 1, device=DEV)
    with pytest.raises(DGLError, match="32 heads"):
        B.fused_gat(g, ft, el, er, 0.2, attn_drop=0.5, seed=1)
    conv = GATConv(16, 4, 64, attn_drop=0.5).to(DEV).train()
    assert not conv._fused_route(g, n)
    y = conv(g, th.randn(n, 16, device=DEV))
    assert y.shape == (n, 64, 4) and th.isfinite(y).all()


def _graph(n_nodes, n_edges, seed):
    src, dst, n = powerlaw(n_nodes, n_edges, seed=seed)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g, n


@pytest.mark.parametrize("nb,p,H,D", [(1, 0.5, 8, 8), (4, 0.5, 8, 8), (1, 0.3, 3, 16),
                                      (1, 0.6, 32, 4), (2, 0.5, 4, 8)])
@pytest.mark.parametrize("in_kernel", [True, False])
def test_gatconv_module_dropout_matches_composition(nb, p, H, D, in_kernel, monkeypatch):
    """The default fused route draws the mask with the module's nn.Dropout: under one
    torch.manual_seed the fused GATConv and the unfused composition (the reference's
    dropout(edge_softmax(...)), which draws on the (E, H, 1) attention) agree within fp32
    tolerance in the output, the input gradient and every parameter gradient -- unblocked
    and with column blocks (the kernels read the keep words through each block's edge
    ids); the route really is the fused one with the module's keep words."""
    from dgl.nn.pytorch.conv import gatconv
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", str(nb))
    monkeypatch.setattr(gatconv, "MODULE_DRAW_IN_KERNEL", in_kernel)
    g, n = _graph(20000, 300000, 21 + nb)
    conv = GATConv(24, D, H, attn_drop=p).to(DEV).train()
    x0 = th.randn(n, 24, device=DEV, generator=th.Generator(device=DEV).manual_seed(2))
    go = th.randn(n, H, D, device=DEV, generator=th.Generator(device=DEV).manual_seed(3))
    calls = []
    orig = B.fused_gat

    def spy(*a, **k):
        calls.append(sorted(k))
        return orig(*a, **k)
    monkeypatch.setattr(B, "fused_gat", spy)
    res = []
    for fused in (True, False):
        conv.use_fused = fused
        conv.zero_grad()
        x = x0.clone().requires_grad_()
        th.manual_seed(11)
        y = conv(g, x)
        y.backward(go)
        res.append((y.detach(), x.grad, conv.fc.weight.grad.clone(), conv.attn_l.grad.clone(),
                    conv.attn_r.grad.clone()))
    assert calls == ([["draw"]] if in_kernel else [["keep", "keep_scale"]])
    (yf, *gf), (yc, *gc) = res
    assert (yc == 0).any()  # dropout happened
    assert th.allclose(yf, yc, rtol=1e-4, atol=1e-5), float((yf - yc).abs().max())
    for a, b, name in zip(gf, gc, ("x", "fc", "attn_l", "attn_r")):
        tol = 1e-4 * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol, (name, float((a - b).abs().max()), tol)
    # a different seed draws a different mask
    conv.use_fused = True
    th.manual_seed(12)
    assert not th.equal(conv(g, x0), yf)


def test_keep_bits_pack():
    """DGLMIGatKeepBits: one word per edge, bit h = (table[e, h] != 0), in the narrowest
    word that holds H (8 / 16 / 32 bits)."""
    gen = th.Generator(device=DEV).manual_seed(4)
    for h in (1, 3, 8, 9, 16, 17, 32):
        t = (th.rand(1001, h, 1, device=DEV, generator=gen) < 0.5).float() * 2.0
        kb = K.gat_keep_bits(t)
        assert kb.dtype == (th.uint8 if h <= 8 else th.int16 if h <= 16 else th.int32)
        bits = kb.cpu().numpy().astype(np.int64) & ((1 << (8 * kb.element_size())) - 1)
        m = (t.reshape(1001, h).cpu().numpy() != 0).astype(np.int64)
        want = (m << np.arange(h, dtype=np.int64)[None, :]).sum(1)
        assert np.array_equal(bits, want)
        # the same words from the boolean mask (DGLMIGatKeepBitsMask), also from a view
        # at an odd byte offset (the 8-head path copies it to an aligned buffer)
        assert th.equal(K.gat_keep_bits(t != 0), kb), h
        flat = th.cat([th.zeros(1, dtype=th.bool, device=DEV), (t != 0).reshape(-1)])
        assert th.equal(K.gat_keep_bits(flat[1:].view(1001, h, 1)), kb), h
    assert K.gat_keep_bits(th.zeros(0, 8, 1, dtype=th.bool, device=DEV)).numel() == 0


@pytest.mark.parametrize("shape", [(13, 1, 1), (1001, 3, 1), (1001, 2, 1), (4099, 8, 1), (70001, 5, 1),
                                   (3_000_001, 2, 1), (5_000_001, 3, 1), (2_000_000, 8, 1),
                                   (1_500_001, 32, 1)])
def test_dropout_draw_matches_native_dropout(shape):
    """dgl.kernel.dropout_draw recomputes torch's fused dropout draw (Philox4x32-10, the
    kernel's launch geometry, vec 4 / 2 / 1 by the element count) -- the mask of
    DGLMIDropoutDrawMask equals torch.native_dropout's from the same generator state, bit
    for bit, and the generator ends at the same offset; at seeds with the offset moved."""
    n = shape[0] * shape[1]
    gen = th.cuda.default_generators[0]
    for seed, pre in ((0, 0), (2 ** 40 + 5, 3)):
        for p in (0.6, 0.1):
            th.manual_seed(seed)
            for _ in range(pre):
                th.native_dropout(th.empty(1000, device=DEV), 0.5, True)
            state = gen.get_state()
            d = K.dropout_draw(DEV, n, p)
            off = gen.get_offset()
            mine = K.dropout_draw_mask(d, n, DEV)
            gen.set_state(state)
            _, ref = th.native_dropout(th.empty(shape, device=DEV), p, True)
            assert gen.get_offset() == off, (shape, seed, p)
            assert th.equal(mine, ref.reshape(-1)), (shape, seed, p, int((mine != ref.reshape(-1)).sum()))
    assert K.dropout_draw_ok(DEV)


def test_gatconv_draw_route_bit_identical_to_mask_route(monkeypatch):
    """The in-kernel draws and torch's own mask packed to keep words give the same fused
    GATConv training step bit for bit (output, gradients) and leave the generator in the
    same state -- unblocked and column-blocked, 8 and 3 heads; and the composition's
    walk-order scale written from the draws (DGLMIDropoutDrawScale) equals nn.Dropout on
    ones gathered into walk order, bit for bit."""
    from dgl.nn.pytorch.conv import gatconv
    # the composition step by step (its fused backward is tested below)
    monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", False)
    for nb, H, fused in ((1, 8, True), (4, 8, True), (1, 3, True), (1, 8, False), (1, 3, False)):
        monkeypatch.setenv("DGLMI_GAT_BLOCKS", str(nb))
        g, n = _graph(20000, 300001, 40 + nb)
        conv = GATConv(24, 8, H, attn_drop=0.45).to(DEV).train()
        conv.use_fused = fused
        x0 = th.randn(n, 24, device=DEV, generator=th.Generator(device=DEV).manual_seed(2))
        go = th.randn(n, H, 8, device=DEV, generator=th.Generator(device=DEV).manual_seed(3))
        res = []
        for in_kernel in (True, False):
            monkeypatch.setattr(gatconv, "MODULE_DRAW_IN_KERNEL", in_kernel)
            conv.zero_grad()
            x = x0.clone().requires_grad_()
            th.manual_seed(5)
            y = conv(g, x)
            y.backward(go)
            res.append((y.detach(), x.grad, conv.fc.weight.grad.clone(), conv.attn_l.grad.clone(),
                        conv.attn_r.grad.clone(), th.cuda.get_rng_state()))
        for a, b in zip(*res):
            assert th.equal(a, b), (nb, H, fused)


@pytest.mark.parametrize("nb,H", [(1, 8), (8, 8), (1, 2), (2, 4)])
def test_composition_dropout_fused_backward(nb, H, monkeypatch):
    """GATConv's composition with attention dropout (use_fused = False): the fused backward
    (GatComposition with the recomputed draws: destination- and source-side walks, no
    slope aggregates) against the step-by-step backward -- the same forward bit for bit,
    the gradients within fp32 tolerance, the generator left in the same state --
    unblocked and column-blocked."""
    from dgl.nn.pytorch.conv import gatconv
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", str(nb))
    g, n = _graph(20000, 300000, 60 + nb)
    conv = GATConv(24, 8, H, attn_drop=0.5).to(DEV).train()
    conv.use_fused = False
    x0 = th.randn(n, 24, device=DEV, generator=th.Generator(device=DEV).manual_seed(2))
    go = th.randn(n, H, 8, device=DEV, generator=th.Generator(device=DEV).manual_seed(3))
    calls = []
    orig = B.gat_composition

    def spy(*a, **k):
        calls.append(k.get("draw") is not None)
        return orig(*a, **k)
    monkeypatch.setattr(B, "gat_composition", spy)
    res = []
    for fused_bwd in (True, False):
        monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", fused_bwd)
        conv.zero_grad()
        x = x0.clone().requires_grad_()
        th.manual_seed(9)
        y = conv(g, x)
        y.backward(go)
        res.append((y.detach(), x.grad, conv.fc.weight.grad.clone(), conv.attn_l.grad.clone(),
                    conv.attn_r.grad.clone(), th.cuda.get_rng_state()))
    assert calls == [True]
    (yf, *gf, sf), (ys, *gs, ss) = res
    assert th.equal(yf, ys) and th.equal(sf, ss)
    for a, b, name in zip(gf, gs, ("x", "fc", "attn_l", "attn_r")):
        tol = 1e-4 * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol, (name, float((a - b).abs().max()), tol)


def test_native_dropout_mask_is_module_draw():
    """GATConv's fused route draws its mask with torch.native_dropout on an uninitialised
    tensor (gatconv.MODULE_DRAW_DTYPE): the same mask, and the same generator state
    after, as the module's nn.Dropout on ones -- the reference's attn_drop draws."""
    from dgl.nn.pytorch.conv import gatconv
    for shape in ((13, 1, 1), (1001, 3, 1), (4099, 8, 1), (70001, 5, 1)):
        th.manual_seed(3)
        ref = th.nn.Dropout(0.6)(th.ones(shape, device=DEV)) != 0
        st = th.cuda.get_rng_state()
        th.manual_seed(3)
        _, m = th.native_dropout(th.empty(shape, device=DEV, dtype=gatconv.MODULE_DRAW_DTYPE), 0.6, True)
        assert th.equal(m, ref), shape
        assert th.equal(th.cuda.get_rng_state(), st), shape


def test_fused_gatconv_ignores_attn_drop(monkeypatch):
    """The reference's FusedGATConv builds attn_drop but calls fused_gat without it
    (fusedGatConv.py:80,152): training output == eval output and equals a
    GATConv without dropout holding the same parameters (eval: bit for bit; training keeps
    the slope aggregates for the backward, the same sums to fp32 rounding)."""
    from dgl.nn.pytorch.conv import FusedGATConv
    g, n = _graph(5000, 60000, 5)
    conv = FusedGATConv(16, 8, 4, attn_drop=0.6).to(DEV)
    plain = GATConv(16, 8, 4).to(DEV)
    plain.load_state_dict(conv.state_dict())
    x = th.randn(n, 16, device=DEV)
    conv.train()
    th.manual_seed(1)
    yt = conv(g, x)
    conv.eval()
    with th.no_grad():
        ye = conv(g, x)
        yp = plain.eval()(g, x)
    assert th.allclose(yt.detach(), ye, rtol=1e-6, atol=1e-7) and th.equal(ye, yp)
    # the unfused fallback does not apply it either
    conv.train()
    conv.use_fused = False
    plain.use_fused = False
    th.manual_seed(1)
    assert th.allclose(conv(g, x), plain.eval()(g, x), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mask", ["module", "hashed"])
def test_gatconv_attn_drop_one(mask):
    """nn.Dropout(1.0) zeroes every attention weight: the output is 0 (no residual) and
    finite gradients; the hashed kernels at p = 1 keep nothing (threshold 2^16, scale 0)
    instead of keeping 1 in 2^16 at an infinite scale."""
    g, n = _graph(3000, 40000, 8)
    conv = GATConv(16, 8, 4, attn_drop=1.0).to(DEV).train()
    conv.attn_drop_mask = mask
    x = th.randn(n, 16, device=DEV, requires_grad=True)
    y = conv(g, x)
    assert th.equal(y, th.zeros_like(y))
    y.sum().backward()
    assert th.isfinite(x.grad).all() and th.isfinite(conv.attn_l.grad).all()
    ft = th.randn(n, 4, 8, device=DEV)
    el, er = th.randn(n, 4, 1, device=DEV), th.randn(n, 4, 1, device=DEV)
    out = B.fused_gat(g, ft, el, er, 0.2, attn_drop=1.0, seed=3)
    assert th.equal(out, th.zeros_like(out))
    assert K.gat_dropout_scale(1.0) == 0.0 and not K.gat_dropout_keep(3, np.arange(100), 4, 1.0).any()


@pytest.mark.parametrize("nb", ["1", "4"])
def test_keep_words_by_edge_id_and_by_position_agree(nb, monkeypatch):
    """DGLMIFusedGatKeep* with the keep words by edge id (a random read per edge in the
    walks) and in the walks' position order (dgl.kernel.gat_keep_walk_order, per column
    block): the same mask, the same kernels -- bit-identical output, slope aggregates and
    gradients."""
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", nb)
    g, n = _graph(20000, 300000, 31)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    H, D = 8, 8
    gen = th.Generator(device=DEV).manual_seed(8)
    ft = th.randn(n, H, D, device=DEV, generator=gen)
    el = th.randn(n, H, 1, device=DEV, generator=gen)
    er = th.randn(n, H, 1, device=DEV, generator=gen)
    go = th.randn(n, H, D, device=DEV, generator=gen)
    t = th.nn.functional.dropout(th.ones(gidx.in_csr.nnz, H, 1, device=DEV), 0.5, True)
    keep = K.gat_keep_bits(t)
    res = []
    for pos in (False, True):
        kin = K.gat_keep_walk_order(gidx, keep, ft, "in") if pos else keep
        kout = K.gat_keep_walk_order(gidx, keep, ft, "out") if pos else keep
        out, mx, sm = (th.empty(n, H, D, device=DEV), th.empty(n, H, device=DEV),
                       th.empty(n, H, device=DEV))
        lf, ls = th.empty(n, H, D, device=DEV), th.empty(n, H, device=DEV)
        K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm, lf, ls, keep=kin, keep_scale=2.0,
                            keep_pos=pos)
        gf, gl, gr = th.empty_like(ft), th.empty_like(el), th.empty_like(er)
        K.fused_gat_backward(gidx, ft, el, er, 0.2, out, mx, sm, go, gf, gl, gr, lf, ls,
                             keep=kout, keep_scale=2.0, keep_pos=pos)
        res.append((out, lf, ls, gf, gl, gr))
    for a, b in zip(*res):
        assert th.equal(a, b)
