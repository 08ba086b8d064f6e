"""Cold-row hints (DGLMIGraph.{in,out}_gather_cols): the hinted copy_u sum
launches (forward on the in-CSR, source gradient on the out-CSR, fused
epilogue) are bit-identical to the unhinted ones and match an fp64 restatement.
The graph is sized so the gathered table reaches the 256 MiB threshold
(2^20 nodes x 64 floats)."""
import os

import pytest
import torch as th

import dgl
from dgl import kernel as K
from dgl.graph_index import device_block_gidx

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def big():
    n, m, f = 1 << 20, 6_000_000, 64
    gen = th.Generator(device=DEV)
    gen.manual_seed(21)
    # skewed sources (some hot rows, many cold) and skewed destinations
    w = th.arange(1, n + 1, device=DEV, dtype=th.float32).pow(-0.9)
    src = th.multinomial(w, m, replacement=True, generator=gen).to(th.int32)
    dst = th.multinomial(w.flip(0), m, replacement=True, generator=gen).to(th.int32)
    x = th.rand(n, f, device=DEV, generator=gen) * 2 - 1
    return n, src, dst, x


def _graph(n, src, dst, hot, max_cold=1.0):
    """The graph with hints at threshold `hot` (0 = none); the cold-share rule is
    relaxed so the marked path is exercised whatever the fixture's share."""
    os.environ["DGLMI_HOT_DEGREE"] = str(hot)
    g = device_block_gidx(n, n, src, dst)
    g.MAX_COLD_SHARE = max_cold
    try:
        g.gather_cols()
    finally:
        os.environ.pop("DGLMI_HOT_DEGREE", None)
    return g


def test_mostly_cold_graph_gets_no_hints():
    """Uniform sources (every row gathered ~6 times): no hot set to protect, so
    the default rule (cold share <= 0.5) leaves the hints off."""
    n, m = 1 << 20, 6_000_000
    gen = th.Generator(device=DEV)
    gen.manual_seed(3)
    src = th.randint(0, n, (m,), device=DEV, generator=gen, dtype=th.int32)
    dst = th.randint(0, n, (m,), device=DEV, generator=gen, dtype=th.int32)
    g = device_block_gidx(n, n, src, dst)
    assert g.gather_cols() == (None, None)


def test_hints_built_and_marked(big):
    n, src, dst, x = big
    g = _graph(n, src, dst, 64)
    ic, oc = g.gather_cols()
    assert ic is not None and oc is not None
    deg_out = th.bincount(src.long(), minlength=n)
    expect = th.where(deg_out[g.in_csr.indices.long()] < 64, g.in_csr.indices | (-2 ** 31),
                      g.in_csr.indices)
    assert th.equal(ic, expect.to(th.int32))
    assert 0.0 < float((ic < 0).float().mean()) < 1.0
    g0 = _graph(n, src, dst, 0)
    assert g0.gather_cols() == (None, None)


def test_hinted_forward_backward_bit_identical(big):
    n, src, dst, x = big
    gh, g0 = _graph(n, src, dst, 64), _graph(n, src, dst, 0)
    row_mul = th.rand(n, device=DEV)
    bias = th.randn(x.shape[1], device=DEV)
    outs = []
    for g in (gh, g0):
        out = th.empty_like(x)
        K.copy_reduce("sum", g, 0, x, out)
        go = th.cos(x[:, :1] * 3.0).expand_as(x).contiguous()
        gx = th.empty_like(x)
        K.backward_copy_reduce("sum", g, 0, x, out, go, gx)
        oe = th.empty_like(x)
        K.copy_reduce("sum", g, 0, x, oe, epilogue=(row_mul, None, bias))
        outs.append((out, gx, oe))
    for a, b in zip(outs[0], outs[1]):
        assert th.equal(a, b)
    # against fp64 gathers
    out = outs[0][0]
    ref = th.zeros(n, x.shape[1], dtype=th.float64, device=DEV).index_add_(
        0, dst.long(), x.double()[src.long()])
    mass = th.zeros_like(ref).index_add_(0, dst.long(), x.double().abs()[src.long()])
    assert bool(((out.double() - ref).abs() <= 1e-4 + 1e-6 * mass).all())


def test_dglgraph_update_all_uses_hints(big, monkeypatch):
    from dgl.graph_index import ImmutableGraphIndex
    monkeypatch.setattr(ImmutableGraphIndex, "MAX_COLD_SHARE", 1.0)
    n, src, dst, x = big
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    g.ndata["h"] = x
    g.update_all(dgl.function.copy_u("h", "m"), dgl.function.sum("m", "o"))
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    assert gidx.gather_cols()[0] is not None
    ref = th.empty_like(x)
    K.copy_reduce("sum", _graph(n, src, dst, 0), 0, x, ref)
    assert th.equal(g.ndata["o"], ref)
