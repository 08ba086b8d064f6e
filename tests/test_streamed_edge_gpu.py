"""u_op_e / e_op_u reductions whose edge operand needs no gradient (fixed edge weights,
R-GCN / GCN norms) stream the operand in walk order on large graphs
(``dgl.backend._StreamedEdgeReduce``): the results and the node gradient must equal the
edge-id walk bit for bit -- the same values in the same summation order -- for every
reducer, both operand orders and broadcast edge operands; an in-place write into the
operand must be seen (the permuted copy is keyed on the version counter).  The edge-id
walk itself is oracle-checked in test_kernels_gpu.py / test_generic_gpu.py."""
import pytest
import torch as th

import dgl
import dgl.function as fn
from dgl import backend as B
from dgl import kernel as K
from graphs import powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def big():
    src, dst, n = powerlaw(200_000, 1_300_000, seed=21)  # past STREAM_EDGE_MIN_EDGES
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g, n, len(src)


def _run(g, msg, red, x, w, streamed, monkeypatch):
    monkeypatch.setenv("DGLMI_STREAM_EDGE", "1" if streamed else "0")
    xr = x.clone().requires_grad_()
    g.ndata["x"] = xr
    g.edata["w"] = w
    g.update_all(msg, red)
    out = g.ndata.pop("h")
    go = th.randn(out.shape, device=DEV, generator=th.Generator(device=DEV).manual_seed(5))
    (gx,) = th.autograd.grad(out, (xr,), go)
    return out.detach(), gx


@pytest.mark.parametrize("op,red,order,shape", [
    ("mul", "sum", "ue", (16,)), ("mul", "mean", "ue", (16,)), ("mul", "max", "ue", (8,)),
    ("add", "min", "eu", (8,)), ("mul", "sum", "eu", (4, 8)), ("sub", "sum", "ue", (4, 8)),
    ("mul", "sum", "ue", (64,))])
def test_streamed_edge_operand_bit_identical(big, op, red, order, shape, monkeypatch):
    g, n, m = big
    gen = th.Generator(device=DEV).manual_seed(3)
    x = th.randn((n,) + shape, device=DEV, generator=gen)
    wshape = (m, 1) if len(shape) == 1 else (m, shape[0], 1)
    w = th.rand(wshape, device=DEV, generator=gen) + 0.5
    msg = getattr(fn, ("u_%s_e" if order == "ue" else "e_%s_u") % op)
    mf = msg("x", "w", "m") if order == "ue" else msg("w", "x", "m")
    rf = getattr(fn, red)("m", "h")
    taken = []
    orig = B._StreamedEdgeReduce.apply

    def spy(*a):
        taken.append(True)
        return orig(*a)
    monkeypatch.setattr(B._StreamedEdgeReduce, "apply", spy)
    # the first use of an operand keeps the edge-id walk; from the second on it streams
    o_first, _ = _run(g, mf, rf, x, w, True, monkeypatch)
    assert not taken
    o1, g1 = _run(g, mf, rf, x, w, True, monkeypatch)
    assert taken, "the streamed route was not taken"
    o0, g0 = _run(g, mf, rf, x, w, False, monkeypatch)
    assert len(taken) == 1
    assert th.equal(o_first, o0)
    assert th.equal(o1, o0)
    assert th.equal(g1, g0)


def test_streamed_edge_operand_sees_inplace_writes(big, monkeypatch):
    g, n, m = big
    x = th.randn(n, 16, device=DEV)
    w = th.rand(m, 1, device=DEV)
    mf, rf = fn.u_mul_e("x", "w", "m"), fn.sum("m", "h")
    for _ in range(2):  # the second call streams (and caches) the operand
        a, _ = _run(g, mf, rf, x, w, True, monkeypatch)
    w.mul_(2.0)  # same storage, new version: the cached permuted copy must be rebuilt
    for _ in range(2):
        b, _ = _run(g, mf, rf, x, w, True, monkeypatch)
    c, _ = _run(g, mf, rf, x, w, False, monkeypatch)
    assert th.equal(b, c)
    assert th.equal(b, 2.0 * a)  # exact: scaling by 2 commutes with fp32 rounding


def test_fresh_operand_per_call_keeps_edge_id_walk(big, monkeypatch):
    """A new operand tensor every call (an attention computed without grad) is never
    permuted, even when the allocator hands it the previous one's address."""
    g, n, m = big
    x = th.randn(n, 16, device=DEV)
    called = []
    orig = B._StreamedEdgeReduce.apply
    monkeypatch.setattr(B._StreamedEdgeReduce, "apply",
                        lambda *a: called.append(1) or orig(*a))
    for i in range(3):
        w = th.full((m, 1), float(i + 1), device=DEV)
        _run(g, fn.u_mul_e("x", "w", "m"), fn.sum("m", "h"), x, w, True, monkeypatch)
        del w
    assert not called


def test_edge_operand_with_grad_keeps_edge_id_walk(big, monkeypatch):
    """An operand that needs a gradient (attention weights) is read by edge id as before,
    and its gradient is the u_dot_v of the fused backward."""
    g, n, m = big
    monkeypatch.setenv("DGLMI_STREAM_EDGE", "1")
    x = th.randn(n, 8, device=DEV)
    w = th.rand(m, 1, device=DEV).requires_grad_()
    called = []
    monkeypatch.setattr(B._StreamedEdgeReduce, "apply", lambda *a: called.append(1))
    g.ndata["x"] = x
    g.edata["w"] = w
    g.update_all(fn.u_mul_e("x", "w", "m"), fn.sum("m", "h"))
    out = g.ndata.pop("h")
    (gw,) = th.autograd.grad(out, (w,), th.ones_like(out))
    assert not called
    src, dst = (th.as_tensor(t).long().to(DEV) for t in g.all_edges())
    ref = x[src].sum(1, keepdim=True)
    assert th.allclose(gw, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("msg,order_by", [("u_mul_e", "dst"), ("copy_e", "dst"), ("u_mul_e", "src")])
def test_dst_sorted_graph_reads_edge_operands_at_positions(msg, order_by, monkeypatch):
    """Edges added in (destination, source) order: the in-CSR's edge ids are its positions
    (DGLMIGraph.eid_identity bit 0, detected once per graph), so edge operands are read
    at the walk position -- the same values in the same order as through the ids."""
    import numpy as np
    src, dst, n = powerlaw(50_000, 400_000, seed=5)
    # (destination, source) order: the in-CSR's own (bit 0); (source, destination): the
    # out-CSR's (bit 1, the node gradient's walk)
    order = np.lexsort((src, dst)) if order_by == "dst" else np.lexsort((dst, src))
    bit = 1 if order_by == "dst" else 2
    src, dst = src[order], dst[order]
    graphs = []
    for detect in ("1", "0"):
        monkeypatch.setenv("DGLMI_EID_IDENTITY", detect)
        g = dgl.DGLGraph()
        g.add_nodes(n)
        g.add_edges(src, dst)
        gidx = g._graph.get_immutable_gidx(DEV)
        assert bool(gidx.eid_identity_bits() & bit) == (detect == "1")
        graphs.append(g)
    gen = th.Generator(device=DEV).manual_seed(9)
    x = th.randn(n, 4, 8, device=DEV, generator=gen)
    e = th.rand(len(src), 4, 1 if msg == "u_mul_e" else 8, device=DEV, generator=gen)
    outs = []
    for g in graphs:
        xr, er = x.clone().requires_grad_(), e.clone().requires_grad_()
        g.ndata["x"], g.edata["e"] = xr, er
        mf = fn.u_mul_e("x", "e", "m") if msg == "u_mul_e" else fn.copy_e("e", "m")
        g.update_all(mf, fn.sum("m", "h"))
        out = g.ndata.pop("h")
        grads = th.autograd.grad(out, (xr, er) if msg == "u_mul_e" else (er,), th.ones_like(out))
        outs.append((out.detach(),) + tuple(grads))
    for a, b in zip(*outs):
        assert th.equal(a, b)


@pytest.mark.parametrize("route", ["dst_sorted", "position_view"])
def test_mapped_u_mul_e_on_identity_edge_ids(route, monkeypatch):
    """A node mapping (lhs_map) on a walk whose edge ids are its positions: the
    per-position weight must be read at each position, not at position 0
    (the identity-id switch to the staged-weight kernel took the mapped
    gather path, which read w[0] for every edge).  Compared with the edge-id walk."""
    import numpy as np
    from dgl import kernel as K
    src, dst, n = powerlaw(40_000, 300_000, seed=13)
    order = np.lexsort((src, dst))
    src, dst = src[order], dst[order]
    m = len(src)
    gen = th.Generator(device=DEV).manual_seed(17)
    D = 16  # D % 4 == 0 and D >= 16: the float4 staged-weight kernel
    x = th.randn(n + 7, D, device=DEV, generator=gen)
    lhs_map = th.randperm(n + 7, device=DEV, generator=gen)[:n].to(th.int32)
    w = th.rand(m, 1, device=DEV, generator=gen) + 0.5
    monkeypatch.setenv("DGLMI_EID_IDENTITY", "0")
    g0 = dgl.DGLGraph()
    g0.add_nodes(n)
    g0.add_edges(src, dst)
    ref = th.zeros(n, D, device=DEV)
    K.binary_op_reduce("sum", "mul", g0._graph.get_immutable_gidx(DEV), "src", "edge", x, w, ref,
                       lhs_map=lhs_map)
    exact = (x[lhs_map.long()][th.as_tensor(src).long().to(DEV)] * w)
    exact = th.zeros(n, D, device=DEV).index_add_(0, th.as_tensor(dst).long().to(DEV), exact)
    assert th.allclose(ref, exact, rtol=1e-4, atol=1e-4)
    if route == "dst_sorted":
        monkeypatch.setenv("DGLMI_EID_IDENTITY", "1")
        g1 = dgl.DGLGraph()
        g1.add_nodes(n)
        g1.add_edges(src, dst)
        gidx = g1._graph.get_immutable_gidx(DEV)
        assert gidx.eid_identity_bits() & 1
        wv = w
    else:
        gidx, wv = g0._graph.get_immutable_gidx(DEV).position_operand(w, "in")
    out = th.zeros(n, D, device=DEV)
    K.binary_op_reduce("sum", "mul", gidx, "src", "edge", x, wv.contiguous(), out, lhs_map=lhs_map)
    assert th.equal(out, ref)


def test_position_operand_cache_drops_with_the_tensor():
    """The position-ordered copy of a constant edge operand is cached by weak reference:
    freeing the operand frees the copy, and clear_operand_cache drops it."""
    import gc
    src, dst, n = powerlaw(30_000, 200_000, seed=3)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(DEV)
    w = th.rand(len(src), 1, device=DEV)
    view, wp = gidx.position_operand(w, "in")
    assert gidx._pos_operands.get("in") is not None
    view2, wp2 = gidx.position_operand(w, "in")
    assert wp2 is wp  # cached
    del w, wp, wp2
    gc.collect()
    assert gidx._pos_operands.get("in") is None
    w = th.rand(len(src), 1, device=DEV)
    gidx.position_operand(w, "out")
    gidx.clear_operand_cache()
    assert not gidx._pos_operands


def test_position_operand_cache_hits_fresh_views():
    """A caller that passes a NEW view of the same constant operand every call
    (_typed_aggregate's ``norm.reshape(E, 1)``) reuses the cached position-ordered copy --
    the weak reference is to the storage owner -- in both directions; an in-place update
    (version bump) misses; freeing the owner drops the entry."""
    import gc
    src, dst, n = powerlaw(20_000, 150_000, seed=4)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(DEV)
    norm = th.rand(len(src), device=DEV)
    _, a = gidx.position_operand(norm.reshape(-1, 1), "in")
    _, b = gidx.position_operand(norm.reshape(-1, 1), "in")
    assert b is a
    _, c = gidx.position_operand(norm.reshape(-1, 1), "out")
    _, d = gidx.position_operand(norm.reshape(-1, 1), "out")
    assert d is c
    assert th.equal(a.flatten(), norm[gidx.in_csr.data.long()])
    norm.mul_(2.0)
    _, e = gidx.position_operand(norm.reshape(-1, 1), "in")
    assert e is not a and th.equal(e.flatten(), norm[gidx.in_csr.data.long()])
    del norm, a, b, c, d, e
    gc.collect()
    assert not gidx._pos_operands


def test_rgcn_flat_norm_copy_dropped_with_the_norm():
    """_flat_norm's contiguous copy of a non-contiguous norm is reused per (tensor,
    version), and dropped from the graph index when the norm is freed."""
    import gc
    from dgl import backend as B
    src, dst, n = powerlaw(5_000, 40_000, seed=5)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gi = g._graph.get_immutable_gidx(DEV)
    base = th.rand(len(src), 2, device=DEV)
    norm = base[:, 1]  # non-contiguous view
    f1 = B._flat_norm(gi, norm)
    f2 = B._flat_norm(gi, base[:, 1])  # a fresh view of the same storage: reused
    assert f2 is f1 and th.equal(f1, norm)
    del norm, base, f1, f2
    gc.collect()
    assert "_rgcn_norm_flat" not in gi.__dict__


@pytest.mark.parametrize("shape", [(1000,), (1000, 3), (1000, 2, 2), (1000, 8, 1), (1000, 4, 16), (1000, 256)])
@pytest.mark.parametrize("idt", [th.int32, th.int64])
def test_gather_rows_matches_indexing(shape, idt):
    """DGLMIGatherRows (the position-order copy of a per-edge operand) equals torch's
    src[index], float4 rows and scalar rows, int32 and int64 indices, repeated and
    out-of-order rows."""
    src = th.randn(*shape, device=DEV)
    idx = th.randint(0, shape[0], (4321,), device=DEV, dtype=idt)
    assert th.equal(K.gather_rows(src, idx), src[idx.long()])
    assert th.equal(K.gather_rows(src, idx, check=True), src[idx.long()])
    assert K.gather_rows(src, idx[:0]).shape == (0,) + tuple(shape[1:])
    from dgl._ffi import DGLError
    for bad in (shape[0], -1):
        with pytest.raises(DGLError, match="out of range"):
            K.gather_rows(src, th.tensor([0, bad], device=DEV, dtype=idt), check=True)
