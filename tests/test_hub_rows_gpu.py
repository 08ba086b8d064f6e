"""Mega-hub rows: one row with millions of entries spans tens of thousands of
chunks, whose carries the fixups fold in segments of kFixSeg by many groups,
the last to finish folding the segment partials in order (csrc/internal.h).
Checked against fp64 torch with the mass-scaled fp32 bound of test_blocks_gpu
(1e-4 + 1e-6 * sum|terms| per row) and exactly for max; deterministic run to
run; both walk directions (in-CSR hub for forwards, out-CSR hub for source
gradients); fused GAT forward and backward against the fp64 dense restatement."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
import dgl.function as fn
from test_fused_gat_gpu import dense_gat

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def star(n, m, hub, reverse=False, seed=0):
    rs = np.random.RandomState(seed)
    other = rs.randint(0, n, m).astype(np.int64)
    hubs = np.full(m, hub, np.int64)
    # a sprinkle of ordinary edges around the hub row
    extra_s, extra_d = rs.randint(0, n, 5000), rs.randint(0, n, 5000)
    src = np.concatenate([hubs if reverse else other, extra_s])
    dst = np.concatenate([other if reverse else hubs, extra_d])
    return src, dst


def _graph(src, dst, n):
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g


def _hub_split(src, dst, n):
    """Edges of rows with > 10^4 entries (reduced row by row: fp64 atomics from
    millions of edges into one row crawl) and the rest (index_add)."""
    s = th.from_numpy(src).to(DEV)
    d = th.from_numpy(dst).to(DEV)
    deg = th.bincount(d, minlength=n)
    hubs = th.nonzero(deg > 10_000).squeeze(1).tolist()
    rest = deg[d] <= 10_000
    return s, d, hubs, rest


def _sum_ref(src, dst, n, x):
    s, d, hubs, rest = _hub_split(src, dst, n)
    xd = x.double()
    exact = th.zeros((n,) + x.shape[1:], dtype=th.float64, device=DEV).index_add_(0, d[rest], xd[s[rest]])
    mass = th.zeros_like(exact).index_add_(0, d[rest], xd[s[rest]].abs())
    for h in hubs:
        rows = xd[s[d == h]]
        exact[h] = rows.sum(0)
        mass[h] = rows.abs().sum(0)
    return exact, mass


@pytest.mark.parametrize("feat", [64, 16, 8, 6])
def test_copy_u_sum_star(feat):
    n, m = 100_000, 3_000_000
    src, dst = star(n, m, hub=777)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(1)
    x = (th.rand(n, feat, device=DEV, generator=gen) * 2 - 1).requires_grad_()
    g.ndata["x"] = x
    g.update_all(fn.copy_u("x", "m"), fn.sum("m", "h"))
    h = g.ndata["h"]
    exact, mass = _sum_ref(src, dst, n, x.detach())
    assert ((h.double() - exact).abs() <= 1e-4 + 1e-6 * mass).all()
    g.update_all(fn.copy_u("x", "m"), fn.sum("m", "h2"))
    assert th.equal(g.ndata["h2"], h)  # deterministic
    go = th.rand(h.shape, device=DEV, generator=gen)
    (gx,) = th.autograd.grad(h, x, go)
    # d/dx[u] = sum over u's out-edges of go[v]: the reverse graph's sum
    gexact, gmass = _sum_ref(dst, src, n, go)
    assert ((gx.double() - gexact).abs() <= 1e-4 + 1e-6 * gmass).all()


@pytest.mark.parametrize("red", ["max", "min"])
def test_copy_u_maxmin_star(red):
    n, m = 100_000, 2_000_000
    src, dst = star(n, m, hub=31)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(2)
    x = th.rand(n, 64, device=DEV, generator=gen)
    g.ndata["x"] = x
    g.update_all(fn.copy_u("x", "m"), getattr(fn, red)("m", "h"))
    s, d, hubs, rest = _hub_split(src, dst, n)
    init = float("-inf") if red == "max" else float("inf")
    ref = th.full((n, 64), init, device=DEV).index_reduce_(0, d[rest], x[s[rest]],
                                                           "amax" if red == "max" else "amin")
    for hb in hubs:
        rows = x[s[d == hb]]
        ref[hb] = rows.amax(0) if red == "max" else rows.amin(0)
    deg = th.bincount(d, minlength=n)
    h = g.ndata["h"]
    assert th.equal(h[deg > 0], ref[deg > 0])


def test_source_gradient_reverse_star():
    """Hub row in the out-CSR: the source-side gradient walk folds its segments."""
    n, m = 100_000, 3_000_000
    src, dst = star(n, m, hub=4242, reverse=True)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(3)
    x = (th.rand(n, 32, device=DEV, generator=gen) * 2 - 1).requires_grad_()
    g.ndata["x"] = x
    g.update_all(fn.copy_u("x", "m"), fn.sum("m", "h"))
    h = g.ndata["h"]
    go = th.rand(h.shape, device=DEV, generator=gen) * 2 - 1
    (gx,) = th.autograd.grad(h, x, go)
    gexact, gmass = _sum_ref(dst, src, n, go)
    assert ((gx.double() - gexact).abs() <= 1e-4 + 1e-6 * gmass).all()


@pytest.mark.parametrize("reverse", [False, True])
def test_fused_gat_star(reverse):
    n, m, H, D = 50_000, 200_000, 4, 4  # the hub row still spans hundreds of chunks
    src, dst = star(n, m, hub=123, reverse=reverse)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(4)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
    er = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
    out = B.fused_gat(g, ft, el, er, 0.2)
    out2 = B.fused_gat(g, ft, el, er, 0.2)
    assert th.equal(out, out2)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gf = th.autograd.grad(out, (ft, el, er), go)
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat(src, dst, n, fd, eld, erd, 0.2)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    for a, b, name in zip(gf, gr, ("ft", "el", "er")):
        err = (a.double() - b).abs().max().item()
        assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), (name, err)


def test_generic_binary_max_star():
    """u_mul_v max reduces on the generic load-balanced kernel (k_lb_fixup)."""
    n, m = 50_000, 1_000_000
    src, dst = star(n, m, hub=99)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(5)
    x = th.rand(n, 3, device=DEV, generator=gen) * 2 - 1
    y = th.rand(n, 3, device=DEV, generator=gen) * 2 - 1
    g.ndata["x"], g.ndata["y"] = x, y
    g.update_all(fn.u_mul_v("x", "y", "m"), fn.max("m", "h"))
    s, d, hubs, rest = _hub_split(src, dst, n)
    ref = th.full((n, 3), float("-inf"), device=DEV).index_reduce_(0, d[rest], x[s[rest]] * y[d[rest]], "amax")
    for hb in hubs:
        ref[hb] = (x[s[d == hb]] * y[hb]).amax(0)
    deg = th.bincount(d, minlength=n)
    assert th.equal(g.ndata["h"][deg > 0], ref[deg > 0])


def test_edge_softmax_star():
    """edge_softmax over a 1 M-edge row: k_sm_fixup's segmented (m, l) merge."""
    from dgl.nn.pytorch import edge_softmax
    n, m = 50_000, 1_000_000
    src, dst = star(n, m, hub=7)
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(6)
    e = (4 * th.randn(len(src), 4, 1, device=DEV, generator=gen)).requires_grad_()
    a = edge_softmax(g, e)
    go = th.randn(a.shape, device=DEV, generator=gen)
    (ge,) = th.autograd.grad(a, e, go)
    d = th.from_numpy(dst).to(DEV)
    hub = d == 7
    ed = e.detach().double()
    ref = th.softmax(ed[hub], dim=0)
    assert th.allclose(a[hub].double(), ref, rtol=1e-4, atol=1e-9)
    gref = ref * (go[hub].double() - (ref * go[hub].double()).sum(0, keepdim=True))
    assert th.allclose(ge[hub].double(), gref, rtol=1e-3, atol=1e-8)
    assert th.allclose(a.sum().double(), th.tensor(float(len(th.unique(d))) * 4, dtype=th.float64,
                                                    device=DEV), rtol=1e-5)
