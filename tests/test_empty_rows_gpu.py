"""Long runs of empty rows (zero in-degree in the walked CSR): a leading, a middle
and a trailing run of thousands of rows, in the in-CSR (forward) and in the
out-CSR (source gradients).  Every load-balanced kernel fills such rows through
its row-parallel share (``fill_empty_rows``, csrc/internal.h) instead of the
chunk that sees the gap.  Parity with the oracle (copy / binary reduce, forward
and gradients, the reference's 1e-4 tolerance, test_kernel.py:292-300) and with
the fp64 dense GAT."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
import dgl.function as fn
from graphs import CODE
from oracle import oracle as O
from test_fused_gat_gpu import dense_gat

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def runs_graph(n=30000, m=120000, seed=5):
    """Destinations in [8000, 11000) and [20000, 20100) only; sources in
    [0, 3000) and [25000, 30000) only: both CSRs have long empty runs."""
    rs = np.random.RandomState(seed)
    dpool = np.concatenate([np.arange(8000, 11000), np.arange(20000, 20100)])
    spool = np.concatenate([np.arange(0, 3000), np.arange(25000, n)])
    dst = dpool[rs.randint(0, len(dpool), m)].astype(np.int64)
    src = spool[rs.randint(0, len(spool), m)].astype(np.int64)
    return src, dst, n


def _graph(src, dst, n):
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g


@pytest.mark.parametrize("red", ["sum", "max", "min", "mean"])
@pytest.mark.parametrize("feat", [(16,), (64,), (3,), (6,), (2, 5)])
def test_copy_u_empty_runs(red, feat):
    src, dst, n = runs_graph()
    rs = np.random.RandomState(7)
    x = rs.uniform(-1, 1, (n,) + feat).astype(np.float32)
    g = _graph(src, dst, n)
    xt = th.from_numpy(x).to(DEV).requires_grad_()
    g.ndata["u"] = xt
    g.update_all(fn.copy_src(src="u", out="m"), getattr(fn, red)(msg="m", out="r"))
    r = g.ndata["r"]
    go = rs.uniform(-1, 1, r.shape).astype(np.float32)
    r.backward(th.from_numpy(go).to(DEV))
    r_out, r_g = O.copy_reduce(red, O.RefGraph(src, dst, n), CODE["u"], x, n, grad_out=go)
    np.testing.assert_allclose(r.detach().cpu().numpy(), r_out, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), r_g, rtol=1e-4, atol=1e-4)
    empty = np.bincount(dst, minlength=n) == 0
    assert empty[:8000].all() and empty[11000:20000].all() and empty[20100:].all()


@pytest.mark.parametrize("lhs,op,rhs,red", [("u", "mul", "e", "sum"), ("u", "add", "v", "max"),
                                            ("e", "sub", "v", "min"), ("u", "dot", "e", "sum")])
def test_binary_empty_runs(lhs, op, rhs, red):
    src, dst, n = runs_graph(m=60000)
    m = len(src)
    rs = np.random.RandomState(9)
    shape = {"u": (n, 4, 3), "v": (n, 4, 3), "e": (m, 4, 3)}
    d = {k: rs.uniform(-1, 1, shape[k]).astype(np.float32) for k in (lhs, rhs)}
    g = _graph(src, dst, n)
    t = {k: th.from_numpy(v).to(DEV).requires_grad_() for k, v in d.items()}
    for k in t:
        (g.edata if k == "e" else g.ndata)[k] = t[k]
    g.update_all(getattr(fn, "%s_%s_%s" % (lhs, op, rhs))(lhs, rhs, "m"), getattr(fn, red)("m", "r"))
    r = g.ndata["r"]
    go = rs.uniform(-1, 1, r.shape).astype(np.float32)
    r.backward(th.from_numpy(go).to(DEV))
    r_out, r_gl, r_gr = O.binary_reduce(red, op, O.RefGraph(src, dst, n), CODE[lhs], CODE[rhs],
                                        d[lhs], d[rhs], n, grad_out=go)
    np.testing.assert_allclose(r.detach().cpu().numpy(), r_out, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(t[lhs].grad.cpu().numpy(), r_gl, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(t[rhs].grad.cpu().numpy(), r_gr, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("H,D", [(8, 8), (2, 16)])
def test_fused_gat_empty_runs(H, D):
    src, dst, n = runs_graph()
    g = _graph(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(4)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
    er = th.randn(n, H, 1, device=DEV, generator=gen).requires_grad_()
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
