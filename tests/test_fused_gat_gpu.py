"""Fused GAT kernel vs the unfused builtin composition (the hack's own
examples/pytorch/gat/fused_gat_unit_test.py strategy: 65,536 nodes, every node
-> hub 0 and hub 1, 8 heads x 8 hidden, slope 0.2) and vs a dense fp64
restatement on a skewed graph with empty rows."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
import dgl.function as fn
from graphs import powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def unfused(g, feat_src, el, er, slope):
    """fused_gat_unit_test.py:37-52 (exp without max subtraction, as the reference)."""
    g = g.local_var()
    g.srcdata.update({"ft": feat_src, "el": el})
    g.dstdata.update({"er": er})
    g.apply_edges(fn.u_add_v("el", "er", "e"))
    e = th.nn.functional.leaky_relu(g.edata.pop("e"), slope)
    g.edata["out"] = th.exp(e)
    g.update_all(fn.copy_e("out", "m"), fn.sum("m", "out_sum"))
    g.apply_edges(fn.e_div_v("out", "out_sum", "out1"))
    g.edata["a"] = g.edata["out1"]
    g.update_all(fn.u_mul_e("ft", "a", "m"), fn.sum("m", "ft"))
    return g.dstdata["ft"]


@pytest.mark.parametrize("H,D", [(8, 8), (4, 16), (1, 4), (2, 32), (8, 128)])
def test_fused_gat_two_hubs(H, D):
    n = 65536 if H * D <= 64 else 8192
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(list(range(n)), 0)
    g.add_edges(list(range(n)), 1)
    th.manual_seed(0)
    ft = th.rand(n, H, D, device=DEV, requires_grad=True)
    el = th.rand(n, H, 1, device=DEV, requires_grad=True)
    er = th.rand(n, H, 1, device=DEV, requires_grad=True)
    r1 = unfused(g, ft, el, er, 0.2)
    r2 = B.fused_gat(g, ft, el, er, 0.2)
    assert th.allclose(r1, r2, rtol=1e-4, atol=1e-5)
    go = th.rand_like(r1)
    g1 = th.autograd.grad(r1, (ft, el, er), go)
    g2 = th.autograd.grad(r2, (ft, el, er), go)
    # grad_er of a hub is sum_e a_e (g_e - delta) over 65,536 in-edges, which cancels
    # to exactly 0 here (all logits > 0, so the leaky derivative is 1): both paths
    # return fp32 noise of ~1e-5 relative to sum |a_e (g_e - delta)| ~ O(1)
    for a, b, name, atol in zip(g1, g2, ("ft", "el", "er"), (1e-5, 1e-5, 1e-4)):
        assert th.allclose(a, b, rtol=1e-3, atol=atol), name


def dense_gat(src, dst, n, ft, el, er, slope):
    s = th.from_numpy(src).to(DEV)
    d = th.from_numpy(dst).to(DEV)
    H = ft.shape[1]
    e = th.nn.functional.leaky_relu(el[s, :, 0] + er[d, :, 0], slope)
    # the shift cancels in the softmax, so it carries no gradient (the amax backward
    # over a star's hub row took ~30 s)
    emax = th.full((n, H), -1e300, dtype=th.float64, device=DEV).index_reduce(0, d, e.detach(), "amax")
    ex = th.exp(e - emax[d])
    den = th.zeros(n, H, dtype=th.float64, device=DEV).index_add(0, d, ex)
    a = ex / den[d]
    return th.zeros(n, H, ft.shape[2], dtype=th.float64, device=DEV).index_add(0, d, ft[s] * a[:, :, None])


@pytest.mark.parametrize("H,D", [(8, 8), (4, 4), (3, 16)])
def test_fused_gat_powerlaw_vs_dense(H, D):
    src, dst, n = powerlaw(20000, 300000, seed=11)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gen = th.Generator(device=DEV).manual_seed(3)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()  # large logits
    er = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    out = B.fused_gat(g, ft, el, er, 0.2)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gf = th.autograd.grad(out, (ft, el, er), go)
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat(src, dst, n, fd, eld, erd, 0.2)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    for a, b, name in zip(gf, gr, ("ft", "el", "er")):
        err = (a.double() - b).abs().max().item()
        assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), (name, err)
    # zero in-degree rows are exact zeros
    zero = th.from_numpy(np.bincount(dst, minlength=n) == 0).to(DEV)
    assert (out[zero] == 0).all()


def test_fused_gatconv_matches_gatconv():
    from dgl.nn.pytorch import GATConv, FusedGATConv
    src, dst, n = powerlaw(5000, 60000, seed=2)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(np.concatenate([src, np.arange(n)]), np.concatenate([dst, np.arange(n)]))
    th.manual_seed(0)
    a = GATConv(32, 8, 8).to(DEV)
    a.use_fused = False
    b = FusedGATConv(32, 8, 8).to(DEV)
    b.load_state_dict(a.state_dict())
    x = th.randn(n, 32, device=DEV)
    ya, yb = a(g, x), b(g, x)
    assert th.allclose(ya, yb, rtol=1e-4, atol=1e-5)
    ya.pow(2).sum().backward()
    yb.pow(2).sum().backward()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert th.allclose(pa.grad, pb.grad, rtol=1e-3, atol=1e-4)


def test_fused_gat_deterministic():
    src, dst, n = powerlaw(20000, 300000, seed=1)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    ft = th.randn(n, 8, 8, device=DEV)
    el = th.randn(n, 8, 1, device=DEV)
    er = th.randn(n, 8, 1, device=DEV)
    assert th.equal(B.fused_gat(g, ft, el, er, 0.2), B.fused_gat(g, ft, el, er, 0.2))


@pytest.mark.parametrize("nb,slopes", [(2, "1"), (4, "1"), (8, "1"), (4, "0"), (8, "0")])
def test_fused_gat_column_blocks_vs_dense(nb, slopes, monkeypatch):
    """Column-blocked launches (DGLMIGraph.num_col_blocks): per-block softmax
    partials merged in block order (forward; with the slope aggregates merged the
    same way), gradients accumulated block by block (backward: the source-side walk
    only, or -- slopes "0" -- the destination-side walk too), against the fp64
    restatement, incl. rows empty in some blocks."""
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", str(nb))
    monkeypatch.setenv("DGLMI_GAT_SLOPES", slopes)
    src, dst, n = powerlaw(20000, 300000, seed=13)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    ib, ob = gidx.col_blocks(nb)
    assert all(c.nnz > 0 for c in ib + ob) and sum(c.nnz for c in ib) == len(src)
    gen = th.Generator(device=DEV).manual_seed(5)
    H, D = 8, 8
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    er = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    out = B.fused_gat(g, ft, el, er, 0.2)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gf = th.autograd.grad(out, (ft, el, er), go)
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat(src, dst, n, fd, eld, erd, 0.2)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    for a, b, name in zip(gf, gr, ("ft", "el", "er")):
        assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), name
    zero = th.from_numpy(np.bincount(dst, minlength=n) == 0).to(DEV)
    assert (out[zero] == 0).all()
    # deterministic (fixed block order)
    assert th.equal(B.fused_gat(g, ft, el, er, 0.2), out)


def test_fused_gat_auto_blocks_match_unblocked(monkeypatch):
    """The automatic rule (dgl.kernel.gat_col_blocks) turns blocking on for a
    >= 32 MiB ft + el table with average in-degree >= 64; results equal the
    unblocked kernels up to summation order."""
    from dgl import kernel as K
    n, m, H, D = 120000, 8_000_000, 8, 8
    gen = th.Generator(device=DEV).manual_seed(9)
    w = th.arange(1, n + 1, device=DEV, dtype=th.float32).pow(-0.4)
    src = th.multinomial(w, m, replacement=True, generator=gen).to(th.int32)
    dst = th.multinomial(w, m, replacement=True, generator=gen).to(th.int32)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
    er = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    assert K.gat_col_blocks(gidx, ft) > 1
    res = []
    for forced in (None, "1"):
        if forced:
            monkeypatch.setenv("DGLMI_GAT_BLOCKS", forced)
        out = B.fused_gat(g, ft, el, er, 0.2)
        grads = th.autograd.grad(out, (ft, el, er), th.cos(out))
        res.append((out,) + grads)
    for a, b in zip(*res):
        assert th.allclose(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("heads,out", [(1, 41), (3, 5), (2, 100)])
def test_gatconv_padded_head_width_matches_unfused(heads, out):
    """Head widths the fused kernel cannot take directly (41 classes, 5, 100) run
    it zero-padded to the next supported width; values and gradients equal the
    unfused composition."""
    from dgl.nn.pytorch import GATConv
    src, dst, n = powerlaw(4000, 50000, seed=6)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(np.concatenate([src, np.arange(n)]), np.concatenate([dst, np.arange(n)]))
    th.manual_seed(0)
    a = GATConv(24, out, heads).to(DEV)
    a.use_fused = False
    b = GATConv(24, out, heads).to(DEV)
    b.load_state_dict(a.state_dict())
    assert b._fused_ok() and b._fused_dim() > out
    x = th.randn(n, 24, device=DEV)
    ya, yb = a(g, x), b(g, x)
    assert yb.shape == (n, heads, out)
    assert th.allclose(ya, yb, rtol=1e-4, atol=1e-5)
    ya.pow(2).sum().backward()
    yb.pow(2).sum().backward()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert th.allclose(pa.grad, pb.grad, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("H,D", [(8, 8), (3, 16), (16, 4)])
def test_fused_gat_edge_position_backward(H, D, monkeypatch):
    """The unblocked backward's three forms: with the forward's slope aggregates
    (default: grad_er = <grad_out, slope_feat> - delta slope_sum from a dense pass), the
    edge-position path (DGLMIGraph.gat_edge_pos: grad_er terms stored in out-CSR order
    by the source-side walk, one gather-sum over the in-CSR) and the destination-side
    walk.  The feature and el gradients are bit-identical across the three (the same
    source-side walk and stats); grad_er differs only in how its sum is formed; all
    match the fp64 restatement, hub rows included."""
    src, dst, n = powerlaw(20000, 300000, seed=29)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gen = th.Generator(device=DEV).manual_seed(9)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    er = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    go = None
    grads = {}
    for slopes, mode in (("1", "1"), ("0", "1"), ("0", "0")):
        monkeypatch.setenv("DGLMI_GAT_SLOPES", slopes)
        monkeypatch.setenv("DGLMI_GAT_EDGE_POS", mode)
        out = B.fused_gat(g, ft, el, er, 0.2)
        if go is None:
            go = th.randn(out.shape, device=DEV, generator=gen)
        grads[slopes + mode] = th.autograd.grad(out, (ft, el, er), go)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    assert getattr(gidx, "_gat_pos", None) is not None  # the edge-position path ran
    for k in ("11", "01"):
        assert th.equal(grads[k][0], grads["00"][0]) and th.equal(grads[k][1], grads["00"][1])
        assert th.allclose(grads[k][2], grads["00"][2], rtol=1e-5, atol=1e-5)
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat(src, dst, n, fd, eld, erd, 0.2)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    for k in ("11", "01"):
        for a, b, name in zip(grads[k], gr, ("ft", "el", "er")):
            assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), (k, name)


@pytest.mark.parametrize("H,D", [(8, 8), (2, 32)])
def test_fused_gat_slope_aggregates_known_answers(H, D):
    """DGLMIFusedGatForwardEx's slope aggregates against their definition in fp64
    (slope_sum = sum_e a_e lrelu'(pre_e), slope_feat = sum_e a_e lrelu'(pre_e) ft[u]),
    with mixed-sign logits so both slopes occur, split rows and empty rows."""
    from dgl import kernel as K
    src, dst, n = powerlaw(20000, 300000, seed=31)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    gen = th.Generator(device=DEV).manual_seed(4)
    ft = th.randn(n, H, D, device=DEV, generator=gen)
    el = 2 * th.randn(n, H, 1, device=DEV, generator=gen)
    er = 2 * th.randn(n, H, 1, device=DEV, generator=gen)
    out, mx, sm = th.empty(n, H, D, device=DEV), th.empty(n, H, device=DEV), th.empty(n, H, device=DEV)
    lf, ls = th.full((n, H, D), float("nan"), device=DEV), th.full((n, H), float("nan"), device=DEV)
    K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm, lf, ls)
    s, d = th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV)
    pre = el.double()[s, :, 0] + er.double()[d, :, 0]
    e = th.nn.functional.leaky_relu(pre, 0.2)
    emax = th.full((n, H), -1e300, dtype=th.float64, device=DEV).index_reduce(0, d, e, "amax")
    ex = th.exp(e - emax[d])
    a = ex / th.zeros(n, H, dtype=th.float64, device=DEV).index_add(0, d, ex)[d]
    slope = th.where(pre > 0, 1.0, 0.2).double()
    ls_ref = th.zeros(n, H, dtype=th.float64, device=DEV).index_add(0, d, a * slope)
    lf_ref = th.zeros(n, H, D, dtype=th.float64, device=DEV).index_add(
        0, d, (a * slope)[:, :, None] * ft.double()[s])
    assert th.allclose(ls.double(), ls_ref, rtol=1e-4, atol=1e-5)
    assert th.allclose(lf.double(), lf_ref, rtol=1e-4, atol=1e-4)
    zero = th.from_numpy(np.bincount(dst, minlength=n) == 0).to(DEV)
    assert (ls[zero] == 0).all() and (lf[zero] == 0).all()
    # the plain forward's outputs are unchanged by keeping them
    out2 = th.empty_like(out)
    K.fused_gat_forward(gidx, ft, el, er, 0.2, out2, th.empty_like(mx), th.empty_like(sm))
    assert th.equal(out, out2)
