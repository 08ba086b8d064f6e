"""Attention dropout inside the fused GAT kernels (DGLMIFusedGatDropout*): GATConv in
training applies ``nn.Dropout`` to the edge softmax (the reference's
``gatconv.py:154``); here the kernels draw the same Bernoulli(1 - p) mask per edge and
head from a hash of a seed and the edge id and scale kept weights by 1 / (1 - p).  The
tests rebuild that mask on the host (``dgl.kernel.gat_dropout_keep``) and check the
output and every gradient against a dense fp64 restatement that applies it to the
softmax -- unblocked and column-blocked -- plus the module routing."""
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
    a = ex / den[d] * (th.from_numpy(keep).to(DEV).double() / (1.0 - p))
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
    """GATConv(attn_drop=0.6) in training takes the fused kernels (no per-edge
    attention tensor), reproducibly under torch.manual_seed; eval mode has no dropout."""
    src, dst, n = powerlaw(5000, 60000, seed=3)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    conv = GATConv(32, 8, 4, attn_drop=0.6).to(DEV)
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
