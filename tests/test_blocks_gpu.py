"""Column blocks on the load-balanced sums (DGLMIGraph.num_col_blocks): one pass
per source block (destination block for the source-side gradient), partial sums
chained through the epilogue addend.  Forced block counts on small graphs and
the automatic rule on a graph that triggers it, against the unblocked kernels
and fp64 restatements; the caller's epilogue (row scale, bias, addend) is kept."""
import pytest
import torch as th

import dgl
import dgl.function as fn
from dgl import kernel as K
from graphs import powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(seed=7, n=6000, m=120000):
    src, dst, n = powerlaw(n, m, seed=seed)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g, src, dst, n


@pytest.mark.parametrize("nb", [2, 4, 8])
@pytest.mark.parametrize("f", [32, 64, 200])
def test_blocked_copy_u_sum_fwd_bwd(nb, f, monkeypatch):
    g, src, dst, n = _graph()
    x = th.randn(n, f, device=DEV, requires_grad=True)
    go = th.randn(n, f, device=DEV)  # fixed upstream gradient (not a function of o)
    res = []
    for blocks in (str(nb), "1"):
        monkeypatch.setenv("DGLMI_SPMM_BLOCKS", blocks)
        gl = g.local_var()
        gl.ndata["x"] = x
        gl.update_all(fn.copy_u("x", "m"), fn.sum("m", "o"))
        o = gl.ndata["o"]
        (gx,) = th.autograd.grad(o, (x,), go)
        res.append((o.detach(), gx))
    s, d = th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV)
    # fp32 sums in a different order differ by up to ~eps * sum|terms| (hub rows
    # of thousands of random-sign terms): bound by that mass, as the other
    # long-sum tests do
    mass_o = th.zeros(n, f, dtype=th.float64, device=DEV).index_add_(0, d, x.double().abs()[s])
    mass_g = th.zeros(n, f, dtype=th.float64, device=DEV).index_add_(0, s, go.double().abs()[d])
    for (a, b), mass in zip(zip(*res), (mass_o, mass_g)):
        assert bool(((a.double() - b.double()).abs() <= 1e-4 + 1e-6 * mass).all())
    ref = th.zeros(n, f, dtype=th.float64, device=DEV).index_add_(0, d, x.double()[s])
    assert bool(((res[0][0].double() - ref).abs() <= 1e-4 + 1e-6 * mass_o).all())
    # deterministic (fixed block order)
    monkeypatch.setenv("DGLMI_SPMM_BLOCKS", str(nb))
    gl = g.local_var()
    gl.ndata["x"] = x.detach()
    gl.update_all(fn.copy_u("x", "m"), fn.sum("m", "o"))
    assert th.equal(gl.ndata["o"], res[0][0])


@pytest.mark.parametrize("nb", [3, 8])
def test_blocked_u_mul_e_bcast_and_epilogue(nb, monkeypatch):
    g, src, dst, n = _graph(seed=9)
    m = len(src)
    H, D = 4, 16
    ft = th.randn(n, H, D, device=DEV, requires_grad=True)
    a = th.rand(m, H, 1, device=DEV, requires_grad=True)
    row_mul = th.rand(n, device=DEV) + 0.5
    bias = th.randn(H * D, device=DEV)
    addend = th.randn(n, H * D, device=DEV)
    go = th.randn(n, H, D, device=DEV)
    res = []
    for blocks in (str(nb), "1"):
        monkeypatch.setenv("DGLMI_SPMM_BLOCKS", blocks)
        gl = g.local_var()
        gl.ndata["ft"] = ft
        gl.edata["a"] = a
        gl.update_all(fn.u_mul_e("ft", "a", "m"), fn.sum("m", "o"))
        o = gl.ndata["o"]
        gft, ga = th.autograd.grad(o, (ft, a), go)
        gidx = g._graph.get_immutable_gidx(th.device(DEV))
        oe = th.empty(n, H * D, device=DEV)
        K.copy_reduce("sum", gidx, 0, ft.detach().reshape(n, H * D), oe,
                      epilogue=(row_mul, None, bias, addend))
        res.append((o.detach(), gft, ga, oe))
    s, d = th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV)
    # blocked and unblocked sums add the same terms in different orders: on hub
    # rows (thousands of in-edges) fp32 reorderings differ by ~eps * sum|term|,
    # so every long sum is bounded by its row mass (as test_blocked_copy_u_sum)
    f64 = ft.detach().double().reshape(n, H * D)
    msg_mass = th.zeros(n, H * D, dtype=th.float64, device=DEV).index_add_(
        0, d, (f64[s].reshape(m, H, D) * a.detach().double()).abs().reshape(m, H * D))
    gft_mass = th.zeros(n, H * D, dtype=th.float64, device=DEV).index_add_(
        0, s, (go.double()[d] * a.detach().double()).abs().reshape(m, H * D))
    cpy_mass = th.zeros(n, H * D, dtype=th.float64, device=DEV).index_add_(0, d, f64.abs()[s])
    epi_mass = cpy_mass * row_mul.double()[:, None] + bias.double().abs() + addend.double().abs()
    masses = (msg_mass, gft_mass, None, epi_mass)
    for x, y, mass in zip(*res, masses):
        x = x.double().reshape(x.shape[0], -1)
        y = y.double().reshape(x.shape)
        if mass is None:  # grad of a: per-edge D-term dots, same order both ways
            assert th.allclose(x, y, rtol=1e-4, atol=1e-4)
        else:
            assert bool(((x - y).abs() <= 1e-4 + 1e-6 * mass).all())
    agg = th.zeros(n, H * D, dtype=th.float64, device=DEV).index_add_(0, d, f64[s])
    ref = agg * row_mul.double()[:, None] + bias.double() + addend.double()
    assert bool(((res[0][3].double() - ref).abs() <= 1e-4 + 1e-6 * epi_mass).all())
    # and against the CPU oracle (the reference's CopyReduce arithmetic) with the
    # epilogue applied on top, at the same mass-scaled bound
    from oracle import oracle as O
    r_out = O.copy_reduce("sum", O.RefGraph(src, dst, n), O.SRC, f64.float().cpu().numpy(), n)
    r_epi = (th.from_numpy(r_out).to(DEV).double() * row_mul.double()[:, None]
             + bias.double() + addend.double())
    assert bool(((res[0][3].double() - r_epi).abs() <= 1e-4 + 1e-6 * epi_mass).all())


def test_auto_spmm_blocks_match_unblocked(monkeypatch):
    """n = 120,000 nodes, 8 M edges, F = 128 (61 MB table, in-degree ~67): the
    rule picks 8 blocks; results equal the unblocked launch."""
    n, m, f = 120000, 8_000_000, 128
    gen = th.Generator(device=DEV).manual_seed(4)
    w = th.arange(1, n + 1, device=DEV, dtype=th.float32).pow(-0.4)
    src = th.multinomial(w, m, replacement=True, generator=gen).to(th.int32)
    dst = th.multinomial(w, m, replacement=True, generator=gen).to(th.int32)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    assert K.spmm_col_blocks(gidx, f) == 8
    x = th.randn(n, f, device=DEV, generator=gen)
    out = th.empty(n, f, device=DEV)
    K.copy_reduce("sum", gidx, 0, x, out)
    monkeypatch.setenv("DGLMI_SPMM_BLOCKS", "1")
    ref = th.empty_like(out)
    K.copy_reduce("sum", gidx, 0, x, ref)
    s64, d64 = src.long(), dst.long()
    mass = th.zeros(n, f, dtype=th.float64, device=DEV).index_add_(0, d64, x.double().abs()[s64])
    assert bool(((out.double() - ref.double()).abs() <= 1e-4 + 1e-6 * mass).all())
