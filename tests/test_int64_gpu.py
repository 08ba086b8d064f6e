"""64-bit graphs on the device: int64 CSR offsets and edge ids, int32 node ids.

The reference switches a graph to int64 ids at 2^31 nodes or edges
(``python/dgl/graph_index.py:941-952``) and then only its CPU kernels run
(``src/kernel/cpu/binary_reduce_sum.cc:15-23``; the CUDA path is int32-only,
``src/kernel/common.h:61-68``).  Here such a graph keeps running on the GPU.

* Small graphs forced to the 64-bit layout (``GraphIndex.asbits(64)``) give results
  bit-identical to the same graph in the int32 layout -- the same kernels and
  summation order, with 64-bit offset and edge-id reads -- for every builtin family:
  copy_u / copy_e / u_mul_e (plain and head-broadcast) sums, max / min / mean and their
  gradients, the generic load-balanced reductions, g-SDDMM, the fused edge softmax,
  GraphConv, GATConv (the fused kernel is int32-only: the composition runs), and
  partial ``pull``; plus the device ingestion against the host COOToCSR / CSRTranspose
  and two reductions against the oracle.
* A graph of 2^31 + 2^20 + 3 edges (4 M nodes) is built on the device (three batches
  of the 64-bit COO -> CSR), and copy_u sum forward / backward and u_mul_e sum are
  checked by size-independent properties (checksums of checksums in fp64), sampled
  rows in fp64, and the sampled rows' CSR contents against the COO sorted by
  (destination, source, edge id).
"""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn
from dgl.graph_index import GraphIndex
from graphs import powerlaw
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pair(src, dst, n):
    g32 = dgl.DGLGraph()
    g32.add_nodes(n)
    g32.add_edges(src, dst)
    g64 = dgl.DGLGraph(g32._graph.asbits(64))
    return g32, g64


def test_device_layout_and_ingestion():
    src, dst, n = powerlaw(3000, 40000, seed=3)
    g32, g64 = _pair(src, dst, n)
    a = g32._graph.get_immutable_gidx(DEV)
    b = g64._graph.get_immutable_gidx(DEV)
    assert a.num_bits == 32 and b.num_bits == 64
    for ca, cb in ((a.in_csr, b.in_csr), (a.out_csr, b.out_csr)):
        assert cb.indptr.dtype == th.int64 and cb.data.dtype == th.int64
        assert cb.indices.dtype == th.int32 and cb.rows.dtype == th.int32
        assert th.equal(ca.indptr.long(), cb.indptr) and th.equal(ca.data.long(), cb.data)
        assert th.equal(ca.indices, cb.indices) and th.equal(ca.rows, cb.rows)
    # device-built 64-bit CSRs (batched stable counting sort) == the host path
    s = th.from_numpy(src).to(DEV, th.int32)
    d = th.from_numpy(dst).to(DEV, th.int32)
    gd = GraphIndex.from_device_coo(s, d, n).asbits(64).get_immutable_gidx(DEV)
    (op, oi, od), (ip, ii, idd) = g32._graph.host_csr()
    for c, (p_, i_, d_) in ((gd.out_csr, (op, oi, od)), (gd.in_csr, (ip, ii, idd))):
        assert c.indptr.dtype == th.int64
        assert np.array_equal(c.indptr.cpu().numpy(), p_)
        assert np.array_equal(c.indices.long().cpu().numpy(), i_)
        assert np.array_equal(c.data.cpu().numpy(), d_)
        assert np.array_equal(c.rows.long().cpu().numpy(),
                              np.repeat(np.arange(n), np.diff(p_)))


def _run(g, feats, fn_call):
    for k, v in feats["n"].items():
        g.ndata[k] = v.detach().clone().requires_grad_()
    for k, v in feats["e"].items():
        g.edata[k] = v.detach().clone().requires_grad_()
    out = fn_call(g)
    go = feats["go"](out)
    leaves = [g.ndata[k] for k in feats["n"]] + [g.edata[k] for k in feats["e"]]
    grads = th.autograd.grad(out, leaves, go, allow_unused=True)
    return out.detach(), [None if x is None else x.detach() for x in grads]


CASES = {
    # (node feature shape, edge feature shape, call)
    "copy_u_sum_F16": ((16,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "copy_u_sum_F5": ((5,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "copy_u_sum_F18": ((18,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "copy_u_sum_F19": ((19,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "copy_u_max_F64": ((64,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.max("m", "o")), g.ndata["o"])[1]),
    "copy_u_min_F8": ((8,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.min("m", "o")), g.ndata["o"])[1]),
    "copy_u_mean_F16": ((16,), None, lambda g: (g.update_all(fn.copy_u("x", "m"), fn.mean("m", "o")), g.ndata["o"])[1]),
    "copy_e_sum_F8": ((4,), (8,), lambda g: (g.update_all(fn.copy_e("w", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "copy_e_max_F4": ((4,), (4,), lambda g: (g.update_all(fn.copy_e("w", "m"), fn.max("m", "o")), g.ndata["o"])[1]),
    "u_mul_e_sum_F32": ((32,), (32,), lambda g: (g.update_all(fn.u_mul_e("x", "w", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "u_mul_e_sum_F4": ((4,), (4,), lambda g: (g.update_all(fn.u_mul_e("x", "w", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "u_mul_e_bcast_H8D8": ((8, 8), (8, 1), lambda g: (g.update_all(fn.u_mul_e("x", "w", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "u_add_v_sum_F6": ((6,), None, lambda g: (g.update_all(fn.u_add_v("x", "x", "m"), fn.sum("m", "o")), g.ndata["o"])[1]),
    "e_div_v_max_F3": ((3,), (3,), lambda g: (g.update_all(fn.e_div_v("w", "x", "m"), fn.max("m", "o")), g.ndata["o"])[1]),
    "u_sub_e_prod_F2": ((2,), (2,), lambda g: (g.update_all(fn.u_sub_e("x", "w", "m"), fn.prod("m", "o")), g.ndata["o"])[1]),
    "u_dot_v_edges_F16": ((16,), None, lambda g: (g.apply_edges(fn.u_dot_v("x", "x", "s")), g.edata["s"])[1]),
    "u_add_v_edges_F8": ((8,), None, lambda g: (g.apply_edges(fn.u_add_v("x", "x", "s")), g.edata["s"])[1]),
    "e_sub_v_edges_F4": ((4,), (4,), lambda g: (g.apply_edges(fn.e_sub_v("w", "x", "s")), g.edata["s"])[1]),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_builtins_bit_identical_to_int32(case):
    nshape, eshape, call = CASES[case]
    src, dst, n = powerlaw(4000, 60000, seed=7)
    g32, g64 = _pair(src, dst, n)
    gen = th.Generator(device=DEV).manual_seed(len(case))
    lo = 0.5 if "div" in case or "prod" in case else -1.0
    feats = {"n": {"x": lo + (1 - lo) * th.rand((n,) + nshape, device=DEV, generator=gen)},
             "e": {} if eshape is None else
                  {"w": lo + (1 - lo) * th.rand((len(src),) + eshape, device=DEV, generator=gen)}}
    go_gen = lambda out: th.randn(out.shape, device=DEV, generator=th.Generator(device=DEV).manual_seed(5))
    feats["go"] = go_gen
    o32, g32s = _run(g32, feats, call)
    o64, g64s = _run(g64, feats, call)
    assert th.equal(o32, o64), case
    for a, b in zip(g32s, g64s):
        assert (a is None) == (b is None)
        if a is not None:
            assert th.equal(a, b), case


@pytest.mark.parametrize("quad", ["0", "1"])
def test_partial_pull_and_softmax_and_modules_bit_identical(monkeypatch, quad):
    from dgl.nn.pytorch import GATConv, GraphConv, edge_softmax
    from dgl.nn.pytorch.conv import gatconv
    # both graphs step by step: the 64-bit graph has no fused walks, so its composition
    # backward runs kernel by kernel; bit identity needs the same on the 32-bit graph
    monkeypatch.setattr(gatconv, "FUSED_COMPOSITION_BACKWARD", False)
    # the composition's edge softmax on the position view: at H <= 4 the 32-bit layout
    # takes the four-values-per-lane walk, the 64-bit layout keeps the one-position walk
    #  -- the same walk (quad "0") gives the same bits, the two walks
    # (quad "1") the same values within fp32 summation-order rounding
    monkeypatch.setenv("DGLMI_SOFTMAX_QUAD", quad)
    src, dst, n = powerlaw(3000, 50000, seed=11)
    g32, g64 = _pair(src, dst, n)
    x = th.randn(n, 16, device=DEV)
    sel = np.unique(np.random.default_rng(1).integers(0, n, 500))
    outs = []
    for g in (g32, g64):
        g.ndata["x"] = x
        g.pull(sel, fn.copy_u("x", "m"), fn.sum("m", "p"))
        logits = th.randn(len(src), 4, 1, device=DEV, generator=th.Generator(device=DEV).manual_seed(2))
        lg = logits.clone().requires_grad_()
        a = edge_softmax(g, lg)
        (ga,) = th.autograd.grad(a, lg, th.ones_like(a))
        th.manual_seed(0)
        gc = GraphConv(16, 8).to(DEV)
        xg = x.clone().requires_grad_()
        y = gc(g, xg)
        (gx,) = th.autograd.grad(y.sum(), xg)
        th.manual_seed(0)
        gat = GATConv(16, 8, 4).to(DEV)
        gat.use_fused = g is g64  # the 64-bit graph must take the composition by itself
        xa = x.clone().requires_grad_()
        z = gat(g, xa)
        (gz,) = th.autograd.grad(z.sum(), xa)
        outs.append((g.ndata["p"], a, ga, y, gx, z, gz))
    for i, (u, v) in enumerate(zip(*outs)):
        if quad == "1" and i >= 5:  # GATConv's output and input gradient
            th.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)
        else:
            assert th.equal(u, v), i


def test_int64_layout_vs_oracle():
    src, dst, n = powerlaw(2000, 30000, seed=13)
    _, g64 = _pair(src, dst, n)
    rng = np.random.default_rng(2)
    x = rng.uniform(-1, 1, (n, 12)).astype(np.float32)
    w = rng.uniform(-1, 1, (len(src), 12)).astype(np.float32)
    g64.ndata["x"] = th.from_numpy(x).to(DEV)
    g64.edata["w"] = th.from_numpy(w).to(DEV)
    g64.update_all(fn.copy_u("x", "m"), fn.sum("m", "a"))
    g64.update_all(fn.u_mul_e("x", "w", "m"), fn.max("m", "b"))
    rg = O.RefGraph(src, dst, n)
    ref_a = O.copy_reduce("sum", rg, O.SRC, x, n)
    ref_b = O.binary_reduce("max", "mul", rg, O.SRC, O.EDGE, x, w, n)
    np.testing.assert_allclose(g64.ndata["a"].cpu().numpy(), ref_a, rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(g64.ndata["b"].cpu().numpy(), ref_b)


def test_graph_of_2_31_edges():
    """2^31 + 2^20 + 3 edges on 4 M nodes, built on the device (about 110 GB of HBM
    while the CSRs are built)."""
    N, F = 1 << 22, 16
    E = (1 << 31) + (1 << 20) + 3
    gen = th.Generator(device=DEV).manual_seed(31)
    src = th.randint(0, N, (E,), dtype=th.int32, device=DEV, generator=gen)
    dst = th.randint(0, N, (E,), dtype=th.int32, device=DEV, generator=gen)
    g = dgl.DGLGraph.from_device_coo(src, dst, N)
    gidx = g._graph.get_immutable_gidx(DEV)
    assert gidx.num_bits == 64 and int(gidx.in_csr.indptr[-1]) == E
    ic, oc = gidx.in_csr, gidx.out_csr
    indeg, outdeg = ic.degrees().double(), oc.degrees().double()
    assert int(indeg.sum()) == E and int(outdeg.sum()) == E

    # sampled rows: CSR contents == the COO's edges into them sorted by (dst, src, eid)
    rows = th.randperm(N, device=DEV, generator=gen)[:64].int().sort().values
    mark = th.zeros(N, dtype=th.bool, device=DEV)
    mark[rows.long()] = True
    step = 1 << 28  # (torch.isin overflows past 2^31 elements)
    eid = th.cat([th.nonzero(mark[dst[b:b + step].long()]).squeeze(1) + b for b in range(0, E, step)])
    s_, d_ = src[eid].long(), dst[eid].long()
    order = th.argsort(s_, stable=True)
    order = order[th.argsort(d_[order], stable=True)]
    st, en = ic.indptr[rows.long()], ic.indptr[rows.long() + 1]
    pos = th.repeat_interleave(st, en - st) + (th.arange(int((en - st).sum()), device=DEV) -
                                              th.repeat_interleave(th.cumsum(en - st, 0) - (en - st), en - st))
    assert th.equal(ic.indices[pos].long(), s_[order]) and th.equal(ic.data[pos], eid[order])

    x = th.rand(N, F, device=DEV, generator=gen) - 0.5
    g.ndata["x"] = x.clone().requires_grad_()
    g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o"))
    out = g.ndata["o"]
    # checksum of checksums: sum_v out[v] = sum_u outdeg(u) x[u]
    lhs = out.detach().double().sum(0)
    rhs = (outdeg[:, None] * x.double()).sum(0)
    mass = (outdeg[:, None] * x.double().abs()).sum(0)
    assert ((lhs - rhs).abs() <= 1e-6 * mass).all()
    # sampled rows in fp64
    seg = th.repeat_interleave(th.arange(len(rows), device=DEV), en - st)
    xs = x.double()[ic.indices[pos].long()]
    ref = th.zeros(len(rows), F, dtype=th.float64, device=DEV).index_add_(0, seg, xs)
    rmass = th.zeros(len(rows), F, dtype=th.float64, device=DEV).index_add_(0, seg, xs.abs())
    assert ((out.detach()[rows.long()].double() - ref).abs() <= 1e-5 + 1e-6 * rmass).all()
    # backward (source gradient on the 64-bit out-CSR): sum_u gx[u] = sum_v indeg(v) go[v]
    go = th.rand(N, F, device=DEV, generator=gen) - 0.5
    (gx,) = th.autograd.grad(out, g.ndata["x"], go)
    lhs = gx.double().sum(0)
    rhs = (indeg[:, None] * go.double()).sum(0)
    mass = (indeg[:, None] * go.double().abs()).sum(0)
    assert ((lhs - rhs).abs() <= 1e-6 * mass).all()
    del gx, go
    # u_mul_e sum with a per-edge weight read by 64-bit edge id
    w = th.rand(E, 1, device=DEV, generator=gen)
    g.edata["w"] = w
    g.update_all(fn.u_mul_e("x", "w", "m"), fn.sum("m", "y"))
    y = g.ndata["y"].detach().double().sum(0)
    ref = th.zeros(F, dtype=th.float64, device=DEV)
    step = 1 << 26
    for b in range(0, E, step):
        ref += (x[src[b:b + step].long()].double() * w[b:b + step].double()).sum(0)
    mass = (outdeg[:, None] * x.double().abs()).sum(0)
    assert ((y - ref).abs() <= 1e-6 * mass).all()
