"""Parity of the per-edge (g-SDDMM) kernels and of the load-balanced generic
reduce on skewed graphs (needs an MI355X).

* Per-edge outputs (reducer "none": ``apply_edges`` with u_add_v, u_dot_v,
  e_sub_v, e_div_v, ...) and per-edge gradients are compared with the oracle
  (``cpu/binary_reduce_impl.h:29-52`` with ReduceNone, the edge branch of
  ``cpu/backward_binary_reduce_impl.h:39-83``) at the reference tolerance 1e-4,
  in both item orders (edge-id order from the COO, and in-CSR positions).
* Node-owned sums (forward reductions and node gradients) run over hub rows
  with 10^4 terms; they are checked against an fp64 restatement with the
  mass-scaled fp32 bound of ``test_kernels_gpu.assert_sum_close``.
* max / min forward values are exact; their gradients go to the tied edges
  (``functor.h:33-44`` + ``BackwardCall``) and match the oracle at 1e-4.
"""
import os
import zlib

import numpy as np
import pytest
import torch as th

import dgl
from oracle import oracle as O
from graphs import CODE, powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def sk():
    src, dst, n = powerlaw(8000, 100000, seed=7)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return src, dst, n, g, O.RefGraph(src, dst, n)


def _feats(n, m, lhs, rhs, op, shape, seed):
    rs = np.random.RandomState(seed)
    rows = {"u": n, "v": n, "e": m}
    lv = rs.uniform(-1, 1, (rows[lhs],) + shape).astype(np.float32)
    rv = rs.uniform(-1, 1, (rows[rhs],) + shape).astype(np.float32)
    if op == "div":
        rv = (np.abs(rv) + 0.5).astype(np.float32) * np.where(rv < 0, -1, 1).astype(np.float32)
    return lv, rv


def _ends(src, dst, t):
    return {"u": src, "v": dst, "e": np.arange(len(src))}[t]


def _edge_terms64(op, L, R, shape):
    """fp64 per-edge op value and its partial derivatives (binary_reduce_common.h:131-213)."""
    m = L.shape[0]
    if op == "dot":
        ln = shape[-1]
        val = (L * R).reshape(m, -1, ln).sum(-1).reshape((m,) + shape[:-1])
        return val, R, L
    val = {"add": L + R, "sub": L - R, "mul": L * R, "div": L / R}[op]
    dl = {"add": np.ones_like(L), "sub": np.ones_like(L), "mul": R, "div": 1 / R}[op]
    dr = {"add": np.ones_like(R), "sub": -np.ones_like(R), "mul": L, "div": -L / (R * R)}[op]
    return val, dl, dr


def _check_node_sum(got, ends, contrib, n):
    """sum_j contrib_j over the edges whose end is the node, against fp64.

    The kernel folds a row's terms in chunks of K <= 512 CSR positions and then
    the <= deg/128 chunk partials in order, so its fp32 error is at most
    (K + deg/128 + 2) * eps * mass (mass = sum_j |contrib_j|).  Same-sign terms
    (add / sub gradients: deg copies of grad_out) approach that bound; the
    reference's single sequential chain would be bounded by deg * eps * mass."""
    flat = contrib.reshape(contrib.shape[0], -1)
    exact = np.zeros((n, flat.shape[1]))
    mass = np.zeros_like(exact)
    np.add.at(exact, ends, flat)
    np.add.at(mass, ends, np.abs(flat))
    deg = np.bincount(ends, minlength=n).astype(np.float64)[:, None]
    got = got.reshape(n, -1).astype(np.float64)
    bound = 1e-4 + (512 + deg / 128 + 2) * 2.0 ** -24 * mass
    err = np.abs(got - exact)
    assert (err <= bound).all(), "max excess %g" % float((err - bound).max())


def _grad_expand(go, shape, op):
    """grad_out per edge broadcast over the dot length."""
    if op == "dot":
        return np.repeat(go[..., None], shape[-1], axis=-1).reshape((go.shape[0],) + shape)
    return go


SHAPES = [(1,), (3,), (8,), (6,), (4, 4), (8, 8), (2, 256), (512,), (3, 5)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "dot"])
@pytest.mark.parametrize("lhs,rhs", [("u", "v"), ("e", "v"), ("u", "e")])
def test_sddmm(sk, lhs, rhs, op, shape):
    if shape in ((2, 256), (512,)) and op in ("add", "sub"):
        # the wide rows' vector path is op-independent; mul / div / dot cover it (the
        # fp64 checks of a 512-wide row over 100 K edges take ~5 s a case)
        pytest.skip("wide rows: covered by mul / div / dot")
    src, dst, n, g, ref = sk
    m = len(src)
    lv, rv = _feats(n, m, lhs, rhs, op, shape, seed=zlib.crc32(repr((lhs, rhs, op, shape)).encode()) % 1000)
    gidx = g._graph.get_immutable_gidx(DEV)
    oshape = shape[:-1] if op == "dot" else shape
    go = np.random.RandomState(3).uniform(-1, 1, (m,) + (oshape or (1,))).astype(np.float32)
    go = go.reshape((m,) + oshape) if oshape else go.reshape(m)
    r_out, r_gl, r_gr = O.binary_reduce("none", op, ref, CODE[lhs], CODE[rhs], lv, rv, m,
                                        grad_out=go.reshape((m,) + (oshape or ())))
    for order in ("coo", "csr"):
        dgl.kernel.set_sddmm_order(order)
        try:
            lt = th.from_numpy(lv).to(DEV).requires_grad_()
            rt = th.from_numpy(rv).to(DEV).requires_grad_()
            out = dgl.backend.binary_reduce("none", op, gidx, CODE[lhs], CODE[rhs], lt, rt, m)
            out.backward(th.from_numpy(go).to(DEV).reshape(out.shape))
        finally:
            dgl.kernel.set_sddmm_order("auto")
        tag = "%s_%s_%s %s %s" % (lhs, op, rhs, shape, order)
        np.testing.assert_allclose(out.detach().cpu().numpy().reshape(r_out.shape), r_out,
                                   rtol=1e-4, atol=1e-4, err_msg=tag)
        # gradients: per-edge operands straight against the oracle, node operands
        # (sums over in/out-edges, hubs included) against fp64
        L64 = lv[_ends(src, dst, lhs)].astype(np.float64)
        R64 = rv[_ends(src, dst, rhs)].astype(np.float64)
        _, dl, dr = _edge_terms64(op, L64, R64, shape)
        ge = _grad_expand(go.reshape((m,) + oshape).astype(np.float64), shape, op)
        for t, grad, r_grad, d in ((lhs, lt.grad, r_gl, dl), (rhs, rt.grad, r_gr, dr)):
            gv = grad.cpu().numpy()
            if t == "e":
                np.testing.assert_allclose(gv, r_grad, rtol=1e-4, atol=1e-4, err_msg=tag + " edge grad")
            else:
                _check_node_sum(gv, _ends(src, dst, t), ge * d, n)


@pytest.mark.parametrize("red", ["sum", "max", "min"])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "dot"])
@pytest.mark.parametrize("lhs,rhs", [("u", "v"), ("e", "v"), ("u", "e")])
@pytest.mark.parametrize("shape", [(4,), (4, 16)], ids=["4", "4x16"])
def test_generic_reduce_skewed(sk, lhs, rhs, op, red, shape):
    """Reductions of the non-specialised message functions to hub rows
    (load-balanced generic kernel) and their gradients."""
    src, dst, n, g, ref = sk
    m = len(src)
    lv, rv = _feats(n, m, lhs, rhs, op, shape, seed=11)
    gidx = g._graph.get_immutable_gidx(DEV)
    lt = th.from_numpy(lv).to(DEV).requires_grad_()
    rt = th.from_numpy(rv).to(DEV).requires_grad_()
    out = dgl.backend.binary_reduce(red, op, gidx, CODE[lhs], CODE[rhs], lt, rt, n)
    go = np.random.RandomState(5).uniform(-1, 1, tuple(out.shape)).astype(np.float32)
    out.backward(th.from_numpy(go).to(DEV))
    r_out, r_gl, r_gr = O.binary_reduce(red, op, ref, CODE[lhs], CODE[rhs], lv, rv, n, grad_out=go)
    got = out.detach().cpu().numpy()
    tag = "%s_%s_%s %s %s" % (lhs, op, rhs, red, shape)
    L64 = lv[_ends(src, dst, lhs)].astype(np.float64)
    R64 = rv[_ends(src, dst, rhs)].astype(np.float64)
    val, dl, dr = _edge_terms64(op, L64, R64, shape)
    if red == "sum":
        _check_node_sum(got, dst, val, n)
        ge = _grad_expand(go[dst].astype(np.float64), shape, op)
        for t, grad, r_grad, d in ((lhs, lt.grad, r_gl, dl), (rhs, rt.grad, r_gr, dr)):
            gv = grad.cpu().numpy()
            if t == "e":
                np.testing.assert_allclose(gv, r_grad, rtol=1e-4, atol=1e-4, err_msg=tag)
            else:
                _check_node_sum(gv, _ends(src, dst, t), ge * d, n)
    else:
        np.testing.assert_array_equal(got, r_out, err_msg=tag)
        np.testing.assert_allclose(lt.grad.cpu().numpy(), r_gl, rtol=1e-4, atol=1e-4, err_msg=tag)
        np.testing.assert_allclose(rt.grad.cpu().numpy(), r_gr, rtol=1e-4, atol=1e-4, err_msg=tag)


def test_coo_order_matches_csr_order_bitwise(sk):
    """Item order changes nothing: every output element is computed by the same
    arithmetic exactly once."""
    src, dst, n, g, _ = sk
    gidx = g._graph.get_immutable_gidx(DEV)
    rs = np.random.RandomState(1)
    u = th.from_numpy(rs.uniform(-1, 1, (n, 8, 8)).astype(np.float32)).to(DEV)
    v = th.from_numpy(rs.uniform(-1, 1, (n, 8, 8)).astype(np.float32)).to(DEV)
    res = []
    for order in ("coo", "csr"):
        os.environ["DGLMI_SDDMM_ORDER"] = order
        try:
            res.append(dgl.backend.binary_reduce("none", "dot", gidx, 0, 1, u, v, len(src)))
        finally:
            os.environ.pop("DGLMI_SDDMM_ORDER", None)
    a, b = res
    assert th.equal(a, b)


def test_apply_edges_full_and_partial():
    """DGLGraph.apply_edges with builtins on all edges (edge-id order via the COO)
    and on a subset (parent-eid subgraph, in-CSR order); untouched rows keep
    their previous value (graph.py apply_edges semantics)."""
    import dgl.function as fn
    src, dst, n = powerlaw(500, 6000, seed=2)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    rs = np.random.RandomState(4)
    u = th.from_numpy(rs.uniform(-1, 1, (n, 4, 8)).astype(np.float32)).to(DEV)
    e = th.from_numpy(rs.uniform(-1, 1, (len(src), 4, 8)).astype(np.float32)).to(DEV)
    g.ndata["h"] = u
    g.edata["w"] = e
    g.apply_edges(fn.u_dot_v("h", "h", "s"))
    s_ref = (u[th.from_numpy(src)] * u[th.from_numpy(dst)]).sum(-1, keepdim=True)
    assert th.allclose(g.edata["s"].reshape(s_ref.shape), s_ref, rtol=1e-5, atol=1e-5)
    g.apply_edges(fn.e_sub_v("w", "h", "d"))
    d_ref = e - u[th.from_numpy(dst)]
    assert th.equal(g.edata["d"], d_ref)
    sub = np.arange(0, len(src), 3)
    g.edata["d2"] = th.zeros_like(e)
    g.apply_edges(fn.u_mul_e("h", "w", "d2"), edges=sub)
    want = th.zeros_like(e)
    want[th.from_numpy(sub)] = u[th.from_numpy(src[sub])] * e[th.from_numpy(sub)]
    assert th.equal(g.edata["d2"], want)


def test_per_edge_and_generic_on_degenerate_graphs():
    """No edges / one edge / isolated nodes: identities, no out-of-range access."""
    for src, dst, n in ((np.zeros(0, np.int64), np.zeros(0, np.int64), 5),
                        (np.array([3]), np.array([1]), 5)):
        g = dgl.DGLGraph()
        g.add_nodes(n)
        if len(src):
            g.add_edges(src, dst)
        gidx = g._graph.get_immutable_gidx(DEV)
        m = len(src)
        u = th.rand(n, 8, device=DEV)
        out = dgl.backend.binary_reduce("none", "add", gidx, 0, 1, u, u, m)
        assert out.shape == (m, 8)
        if m:
            assert th.equal(out[0], u[3] + u[1])
        for red, ident in (("sum", 0.0), ("max", -3.402823466e38), ("min", 3.402823466e38)):
            r = dgl.backend.binary_reduce(red, "sub", gidx, 0, 1, u, u, n)
            rows = [v for v in range(n) if v not in set(dst.tolist())]
            assert bool((r[rows] == ident).all()), red
            if m:
                assert th.equal(r[1], u[3] - u[1])
