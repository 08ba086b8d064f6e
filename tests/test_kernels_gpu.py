"""Parity of the HIP kernels with the CPU oracle (needs an MI355X).

Every builtin message x reducer x broadcast x {full, partial} combination of
tests/compute/test_kernel.py runs through DGLGraph -> dgl.backend -> the C ABI
-> libdglmi.so and is compared with the oracle (forward and gradients) at the
reference's tolerance (rtol = atol = 1e-4, 1e-2 for prod; test_kernel.py:292-300).
max / min forward values are exact (no rounding is involved).
"""
import itertools

import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn
from oracle import oracle as O
from graphs import CODE, binary_case_features, er_graph, g20, powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(src, dst, n):
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g


def _run_binary(g, d, lhs, rhs, op, red, nid=None):
    feats = {k: th.from_numpy(v).to(DEV).requires_grad_() for k, v in d.items()}
    g.ndata["u"] = feats["u"]
    g.ndata["v"] = feats["v"]
    g.edata["e"] = feats["e"]
    msg = getattr(fn, "%s_%s_%s" % (lhs, op, rhs))(lhs, rhs, "m")
    if nid is None:
        g.update_all(msg, getattr(fn, red)("m", "r1"))
    else:
        g.pull(nid, msg, getattr(fn, red)("m", "r1"))
    r1 = g.ndata.pop("r1")
    r1.sum().backward()
    return (r1.detach().cpu().numpy(), feats[lhs].grad.cpu().numpy(),
            feats[rhs].grad.cpu().numpy())


@pytest.mark.parametrize("lhs,rhs", [(a, b) for a, b in itertools.product("uve", "uve") if a != b])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "dot"])
def test_all_binary_builtins(lhs, rhs, op):
    src, dst, n = g20()
    m = len(src)
    ref = O.RefGraph(src, dst, n)
    nid = np.array([0, 1, 4, 5, 7, 12, 14, 15, 18, 19])
    for red in ["sum", "max", "min", "prod", "mean"]:
        for bc in ["none", lhs, rhs]:
            for partial in (False, True):
                d = binary_case_features(n, m, lhs, rhs, op, bc)
                g = _graph(src, dst, n)
                out, gl, gr = _run_binary(g, d, lhs, rhs, op, red, nid if partial else None)
                go = np.ones((n,) + out.shape[1:], np.float32)
                if partial:
                    mask = np.zeros(n, bool)
                    mask[nid] = True
                    go[~mask] = 0
                r_out, r_gl, r_gr = O.binary_reduce(red, op, ref, CODE[lhs], CODE[rhs], d[lhs],
                                                    d[rhs], n, grad_out=go)
                tol = 1e-2 if red == "prod" else 1e-4
                msg = "%s_%s_%s %s bcast=%s partial=%s" % (lhs, op, rhs, red, bc, partial)
                rows = nid if partial else slice(None)
                np.testing.assert_allclose(out[rows], r_out[rows], rtol=tol, atol=tol, err_msg=msg)
                np.testing.assert_allclose(gl, r_gl, rtol=tol, atol=tol, err_msg=msg + " lhs grad")
                np.testing.assert_allclose(gr, r_gr, rtol=tol, atol=tol, err_msg=msg + " rhs grad")


@pytest.mark.parametrize("red", ["sum", "max", "mean"])
@pytest.mark.parametrize("target", ["u", "e"])
@pytest.mark.parametrize("partial", [False, True])
def test_copy_reduce(red, target, partial):
    """test_kernel.py:77-197: copy_src / copy_edge x {sum, max, mean}."""
    src, dst, n = er_graph(100, 0.1, seed=1)
    m = len(src)
    rs = np.random.RandomState(31)
    x = rs.uniform(-1, 1, ((n if target == "u" else m), 5, 3, 4)).astype(np.float32)
    g = _graph(src, dst, n)
    xt = th.from_numpy(x).to(DEV).requires_grad_()
    if target == "u":
        g.ndata["u"] = xt
        msg = fn.copy_src(src="u", out="m")
    else:
        g.edata["e"] = xt
        msg = fn.copy_edge(edge="e", out="m")
    nid = np.arange(0, 100, 2)
    if partial:
        g.pull(nid, msg, getattr(fn, red)(msg="m", out="r1"))
    else:
        g.update_all(msg, getattr(fn, red)(msg="m", out="r1"))
    r1 = g.ndata["r1"]
    r1.sum().backward()
    go = np.ones((n, 5, 3, 4), np.float32)
    if partial:
        mask = np.zeros(n, bool)
        mask[nid] = True
        go[~mask] = 0
    ref = O.RefGraph(src, dst, n)
    r_out, r_g = O.copy_reduce(red, ref, CODE[target], x, n, grad_out=go)
    rows = nid if partial else slice(None)
    np.testing.assert_allclose(r1.detach().cpu().numpy()[rows], r_out[rows], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), r_g, rtol=1e-4, atol=1e-4)


def test_golden_vectors():
    """GPU against the committed golden vectors of the oracle."""
    import os
    import make_golden
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "kernel_g20.npz"))
    src, dst, n = z["src"], z["dst"], 20
    g = _graph(src, dst, n)
    for lhs, op, rhs, red, bc in make_golden.CASES:
        name = "%s_%s_%s_%s_%s" % (lhs, op, rhs, red, bc)
        gidx = g._graph.get_immutable_gidx(DEV)
        out_rows = len(src) if red == "none" else n
        t = lambda k: th.from_numpy(z[name + "/" + k]).to(DEV)
        if op == "use_lhs":
            x = t("x").requires_grad_()
            out = dgl.backend.copy_reduce(red, gidx, CODE[lhs], x, out_rows)
            out.backward(t("grad_out"))
            pairs = [(out, "out"), (x.grad, "grad_x")]
        else:
            l, r = t("lhs").requires_grad_(), t("rhs").requires_grad_()
            out = dgl.backend.binary_reduce(red, op, gidx, CODE[lhs], CODE[rhs], l, r, out_rows)
            out.backward(t("grad_out"))
            pairs = [(out, "out"), (l.grad, "grad_lhs"), (r.grad, "grad_rhs")]
        for val, k in pairs:
            np.testing.assert_allclose(val.detach().cpu().numpy(), z[name + "/" + k], rtol=1e-4,
                                       atol=1e-4, err_msg=name + "/" + k)


def _weighted_sums(csr, x, w=None):
    """fp64 sum_j w_j x[col_j] and its mass sum_j |w_j x[col_j]| per row (scipy)."""
    import scipy.sparse as sp
    indptr, indices, eids = csr
    n = len(indptr) - 1
    x2 = x.reshape(x.shape[0], -1).astype(np.float64)
    if w is None:
        A = sp.csr_matrix((np.ones(len(indices)), indices, indptr), shape=(n, x.shape[0]))
        return A @ x2, A @ np.abs(x2)
    # w: per-edge weights (E, H) broadcast over the trailing dim of x (N, H, D)
    H = w.shape[1]
    x3 = x.reshape(x.shape[0], H, -1).astype(np.float64)
    ex = np.zeros((n, H, x3.shape[2]))
    ms = np.zeros_like(ex)
    for h in range(H):
        wh = w[eids, h].astype(np.float64)
        A = sp.csr_matrix((wh, indices, indptr), shape=(n, x.shape[0]))
        Aa = sp.csr_matrix((np.abs(wh), indices, indptr), shape=(n, x.shape[0]))
        ex[:, h] = A @ x3[:, h]
        ms[:, h] = Aa @ np.abs(x3[:, h])
    return ex.reshape(n, -1), ms.reshape(n, -1)


def assert_sum_close(got, ref32, csr, x, w=None):
    """fp32 sums over rows with up to 10^4-10^5 terms: the oracle's sequential fp32
    order and the kernel's chunked order both carry rounding error that grows with
    the row's mass sum|term|.  Both are checked against an fp64 restatement with a
    bound of 1e-4 + 1e-6 * mass (fp32 eps = 6e-8; sequential worst case ~ n * eps),
    and the kernel against the oracle at the reference tolerance 1e-4 on rows whose
    mass is small (< 100), i.e. everywhere the reference's own tolerance is meaningful."""
    exact, mass = _weighted_sums(csr, x, w)
    exact = exact.reshape(got.shape)
    mass = mass.reshape(got.shape)
    bound = 1e-4 + 1e-6 * mass
    # the oracle's single sequential fp32 chain may drift further on 10^5-term rows
    assert (np.abs(ref32 - exact) <= 1e-4 + 1e-5 * mass).all(), "oracle outside the fp32 bound"
    assert (np.abs(got - exact) <= bound).all(), float(np.abs(got - exact).max())
    small = mass < 100
    np.testing.assert_allclose(got[small], ref32[small], rtol=1e-4, atol=1e-4)


# --------------------------------------------------------------------------
# load-balanced path: skewed graphs, hub rows split over many chunks
# --------------------------------------------------------------------------
@pytest.fixture(scope="module")
def plaw():
    src, dst, n = powerlaw(20000, 400000, seed=5)
    return src, dst, n, _graph(src, dst, n), O.RefGraph(src, dst, n)


# 10, 18, 30, 33, 511, 601, 602, 1022, 2046: rows that are not a multiple of 4 floats
# (float2 / single-float slots of the load-balanced kernel; 602 = Reddit's F_in);
# 2048: 8 float4 slots per lane; 1433 (Cora's F_in): the generic kernel
@pytest.mark.parametrize("F", [1, 2, 3, 4, 7, 8, 12, 16, 20, 64, 128, 256, 512, 1024, 6, 10,
                               18, 30, 33, 511, 601, 602, 1022, 2046, 2048, 1433])
@pytest.mark.parametrize("red", ["sum", "max", "min"])
def test_copy_u_powerlaw(plaw, F, red):
    src, dst, n, g, ref = plaw
    x = np.random.RandomState(F).uniform(-1, 1, (n, F)).astype(np.float32)
    gidx = g._graph.get_immutable_gidx(DEV)
    xt = th.from_numpy(x).to(DEV).requires_grad_()
    out = dgl.backend.copy_reduce(red, gidx, 0, xt, n)
    go = np.random.RandomState(1).uniform(-1, 1, (n, F)).astype(np.float32)
    out.backward(th.from_numpy(go).to(DEV))
    r_out, r_g = O.copy_reduce(red, ref, O.SRC, x, n, grad_out=go)
    o = out.detach().cpu().numpy()
    if red == "sum":
        assert_sum_close(o, r_out, ref.in_csr, x)
        assert_sum_close(xt.grad.cpu().numpy(), r_g, ref.out_csr, go)
    else:
        np.testing.assert_array_equal(o, r_out)
        # gradient goes to every tied (== max) edge: few terms per source row
        np.testing.assert_allclose(xt.grad.cpu().numpy(), r_g, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("F", [1, 8, 16, 64, 256, 18, 33, 602])
def test_copy_e_powerlaw(plaw, F):
    src, dst, n, g, ref = plaw
    m = len(src)
    x = np.random.RandomState(F).uniform(-1, 1, (m, F)).astype(np.float32)
    gidx = g._graph.get_immutable_gidx(DEV)
    for red in ("sum", "max"):
        out = dgl.backend.copy_reduce(red, gidx, 2, th.from_numpy(x).to(DEV), n)
        r_out = O.copy_reduce(red, ref, O.EDGE, x, n)
        if red == "sum":
            ip, _, eids = ref.in_csr
            # edge data gathered by eid: a CSR whose "columns" are the edge ids
            assert_sum_close(out.cpu().numpy(), r_out, (ip, eids, eids), x)
        else:
            np.testing.assert_array_equal(out.cpu().numpy(), r_out)


@pytest.mark.parametrize("H,D", [(8, 8), (4, 16), (1, 64), (8, 3), (2, 4), (8, 1), (1, 1),
                                 (4, 6), (2, 9), (7, 86)])
def test_u_mul_e_bcast_powerlaw(plaw, H, D):
    """GAT aggregation: (N, H, D) x (E, H, 1) -> sum, forward and both gradients."""
    src, dst, n, g, ref = plaw
    m = len(src)
    rs = np.random.RandomState(H * D)
    ft = rs.uniform(-1, 1, (n, H, D)).astype(np.float32)
    a = rs.uniform(0, 1, (m, H, 1)).astype(np.float32)
    gidx = g._graph.get_immutable_gidx(DEV)
    ftt = th.from_numpy(ft).to(DEV).requires_grad_()
    at = th.from_numpy(a).to(DEV).requires_grad_()
    out = dgl.backend.binary_reduce("sum", "mul", gidx, 0, 2, ftt, at, n)
    go = rs.uniform(-1, 1, (n, H, D)).astype(np.float32)
    out.backward(th.from_numpy(go).to(DEV))
    r_out, r_gl, r_gr = O.binary_reduce("sum", "mul", ref, 0, 2, ft, a, n, grad_out=go)
    assert_sum_close(out.detach().cpu().numpy(), r_out, ref.in_csr, ft, a.reshape(m, H))
    np.testing.assert_allclose(ftt.grad.cpu().numpy(), r_gl, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(at.grad.cpu().numpy(), r_gr, rtol=1e-4, atol=2e-4)


def test_u_mul_e_same_shape(plaw):
    src, dst, n, g, ref = plaw
    m = len(src)
    rs = np.random.RandomState(3)
    x = rs.uniform(-1, 1, (n, 32)).astype(np.float32)
    w = rs.uniform(-1, 1, (m, 32)).astype(np.float32)
    gidx = g._graph.get_immutable_gidx(DEV)
    out = dgl.backend.binary_reduce("sum", "mul", gidx, 0, 2, th.from_numpy(x).to(DEV),
                                    th.from_numpy(w).to(DEV), n).cpu().numpy()
    r = O.binary_reduce("sum", "mul", ref, 0, 2, x, w, n)
    ip, idx, eids = ref.in_csr
    msg = x[idx].astype(np.float64) * w[eids]
    exact = np.add.reduceat(np.vstack([msg, np.zeros((1, 32))]), np.minimum(ip[:-1], len(idx)), axis=0)
    exact[ip[:-1] == ip[1:]] = 0
    mass = np.add.reduceat(np.vstack([np.abs(msg), np.zeros((1, 32))]), np.minimum(ip[:-1], len(idx)), axis=0)
    mass[ip[:-1] == ip[1:]] = 0
    bound = 1e-4 + 1e-6 * mass
    assert (np.abs(out - exact) <= bound).all() and (np.abs(r - exact) <= bound).all()


def test_deterministic(plaw):
    """Owner-computes + ordered carry fold: bitwise identical across runs."""
    src, dst, n, g, ref = plaw
    x = th.randn(n, 64, device=DEV)
    gidx = g._graph.get_immutable_gidx(DEV)
    a = dgl.backend.copy_reduce("sum", gidx, 0, x, n)
    b = dgl.backend.copy_reduce("sum", gidx, 0, x, n)
    assert th.equal(a, b)


def test_single_hub_and_gaps():
    """All edges into one row (spans every chunk), leading/trailing empty rows."""
    n, m = 5000, 200000
    rng = np.random.default_rng(2)
    src = rng.integers(0, n, m)
    dst = np.full(m, 2500)
    dst[:10] = 3  # a small row before the hub
    g = _graph(src, dst, n)
    ref = O.RefGraph(src, dst, n)
    x = rng.uniform(-1, 1, (n, 64)).astype(np.float32)
    gidx = g._graph.get_immutable_gidx(DEV)
    for red in ("sum", "max", "min"):
        out = dgl.backend.copy_reduce(red, gidx, 0, th.from_numpy(x).to(DEV), n).cpu().numpy()
        r = O.copy_reduce(red, ref, O.SRC, x, n)
        if red == "sum":
            assert_sum_close(out, r, ref.in_csr, x)
        else:
            np.testing.assert_array_equal(out, r)


def test_empty_graph_and_isolated():
    """Edgeless graph: update_all downgrades to apply_nodes and writes no reduce
    field (scheduler.py:216-222); the kernel itself still identity-fills every row
    (binary_reduce_common.h:444-485), and so do isolated rows of a graph with edges."""
    g = dgl.DGLGraph()
    g.add_nodes(7)
    g.ndata["h"] = th.ones(7, 16, device=DEV)
    g.update_all(fn.copy_u("h", "m"), fn.sum("m", "s"))
    assert "s" not in g.ndata
    gidx = g._graph.get_immutable_gidx(DEV)
    assert th.equal(dgl.backend.copy_reduce("sum", gidx, 0, g.ndata["h"], 7),
                    th.zeros(7, 16, device=DEV))
    assert (dgl.backend.copy_reduce("max", gidx, 0, g.ndata["h"], 7)
            == -3.4028234663852886e38).all()
    g = dgl.DGLGraph()
    g.add_nodes(7)
    g.add_edges([0], [1])
    g.ndata["h"] = th.ones(7, 16, device=DEV)
    g.update_all(fn.copy_u("h", "m"), fn.sum("m", "s"))
    assert th.equal(g.ndata["s"][1], th.ones(16, device=DEV))
    assert th.equal(g.ndata["s"][th.tensor([0, 2, 3, 4, 5, 6])], th.zeros(6, 16, device=DEV))
    g.update_all(fn.copy_u("h", "m"), fn.max("m", "s"))
    assert (g.ndata["s"][th.tensor([0, 2, 3, 4, 5, 6])] == -3.4028234663852886e38).all()


def test_rejects_cpu_tensors():
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 1], [1, 2])
    g.ndata["h"] = th.ones(3, 4)
    with pytest.raises(dgl.DGLError):
        g.update_all(fn.copy_u("h", "m"), fn.sum("m", "s"))


def test_device_ingest_bit_exact():
    """Device COO->CSR (radix sort) == host counting sort == reference KATs."""
    from dgl.graph_index import GraphIndex
    src, dst, n = powerlaw(30000, 500000, seed=9)
    host = GraphIndex(n)
    host.add_edges(src, dst)
    dev = GraphIndex.from_device_coo(th.from_numpy(src).to(DEV, th.int32),
                                     th.from_numpy(dst).to(DEV, th.int32), n)
    a = host.get_immutable_gidx(DEV)
    b = dev.get_immutable_gidx(DEV)
    for x, y in ((a.in_csr, b.in_csr), (a.out_csr, b.out_csr)):
        for k in ("indptr", "indices", "data", "rows"):
            assert th.equal(getattr(x, k), getattr(y, k)), k
    ref = O.RefGraph(src, dst, n)
    np.testing.assert_array_equal(b.in_csr.indptr.cpu().numpy(), ref.in_csr[0])
    np.testing.assert_array_equal(b.in_csr.indices.cpu().numpy(), ref.in_csr[1])
    np.testing.assert_array_equal(b.in_csr.data.cpu().numpy(), ref.in_csr[2])


@pytest.mark.parametrize("F", [4, 7, 64, 12, 128, 18, 33, 602])
def test_fused_epilogue(plaw, F):
    """copy_u_sum with every epilogue term (row_mul, row_div, bias, addend), on the
    load-balanced kernels (hub rows split across chunks) and on the generic
    fallback (a mapped output), against torch on the plain sum."""
    from dgl import kernel as K
    src, dst, n, g, _ = plaw
    gidx = g._graph.get_immutable_gidx(DEV)
    gen = th.Generator(device=DEV).manual_seed(F)
    x = th.rand(n, F, generator=gen, device=DEV) - 0.5
    mul = th.rand(n, generator=gen, device=DEV) + 0.5
    div = th.rand(n, generator=gen, device=DEV) + 0.5
    bias = th.rand(F, generator=gen, device=DEV)
    add = th.rand(n, F, generator=gen, device=DEV)
    plain = th.empty(n, F, device=DEV)
    K.copy_reduce("sum", gidx, 0, x, plain)
    want = ((plain * mul[:, None]) / div[:, None] + bias) + add
    out = th.empty(n, F, device=DEV)
    K.copy_reduce("sum", gidx, 0, x, out, epilogue=(mul, div, bias, add))
    assert th.equal(out, want)
    # generic path: the same through an identity out_map
    omap = th.arange(n, dtype=th.int32, device=DEV)
    out2 = th.empty(n, F, device=DEV)
    K.copy_reduce("sum", gidx, 0, x, out2, out_map=omap, epilogue=(mul, div, bias, add))
    # a different summation order over hub rows of 10^4 terms: both against fp64
    # with the mass bound of assert_sum_close (1e-4 + 1e-6 * sum|term|, scaled by
    # the epilogue's row factor)
    s64 = th.as_tensor(src, device=DEV).long()
    d64 = th.as_tensor(dst, device=DEV).long()
    exact = th.zeros(n, F, dtype=th.float64, device=DEV).index_add_(0, d64, x.double()[s64])
    mass = th.zeros(n, F, dtype=th.float64, device=DEV).index_add_(0, d64, x.double()[s64].abs())
    scale = (mul / div).double()[:, None]
    exact = exact * scale + bias.double() + add.double()
    bound = 1e-4 + 1e-6 * mass * scale
    assert ((want.double() - exact).abs() <= bound).all()
    assert ((out2.double() - exact).abs() <= bound).all(), float((out2 - want).abs().max())
    with pytest.raises(dgl.DGLError):
        K.copy_reduce("max", gidx, 0, x, out, epilogue=(mul, None, None))
    with pytest.raises(dgl.DGLError):
        K.copy_reduce("sum", gidx, 0, x, out, epilogue=(None, None, None, out))


_SPECIAL = None


def _special():
    global _SPECIAL
    if _SPECIAL is None:
        import json
        import os
        p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "special_values.json")
        _SPECIAL = json.load(open(p))
    return _SPECIAL


@pytest.mark.parametrize("red", ["sum", "max", "min"])
def test_special_values_known_answers(red):
    """NaN / +-inf messages and zero-in-degree rows through update_all: the
    kernels keep std::max / std::min semantics (a NaN message never replaces the
    accumulator, functor.h:33,44), the identity fill and the tie-mask gradient.
    Known answers (tests/golden/make_special.py) and the oracle, bit for bit."""
    d = _special()
    g = _graph(np.array(d["src"]), np.array(d["dst"]), d["n"])
    x = th.tensor(d["x"], dtype=th.float32, device=DEV, requires_grad=True)
    g.ndata["x"] = x
    g.update_all(fn.copy_u("x", "m"), getattr(fn, red)("m", "o"))
    o = g.ndata["o"]
    o.backward(th.ones_like(o))
    want_o = np.array(d["cases"][red]["out"], np.float32)
    want_g = np.array(d["cases"][red]["grad_x"], np.float32)
    np.testing.assert_array_equal(o.detach().cpu().numpy(), want_o)
    np.testing.assert_array_equal(x.grad.cpu().numpy(), want_g)
    xr = np.array(d["x"], np.float32)
    r_o, r_g = O.copy_reduce(red, O.RefGraph(np.array(d["src"]), np.array(d["dst"]), d["n"]),
                             O.SRC, xr, d["n"], grad_out=np.ones_like(xr))
    np.testing.assert_array_equal(o.detach().cpu().numpy(), r_o)
    np.testing.assert_array_equal(x.grad.cpu().numpy(), r_g)


@pytest.mark.parametrize("fused", [True, False])
def test_special_values_edge_softmax(fused, monkeypatch):
    """All-masked (-inf), NaN and +inf logits: the fused kernel pair and the
    decomposition both give the reference decomposition's values (NaN rows
    included, softmax.py:33-78)."""
    from dgl.nn.pytorch import softmax as S
    monkeypatch.setattr(S, "FUSED", fused)
    d = _special()
    sm = d["softmax"]
    g = _graph(np.array(sm["src"]), np.array(sm["dst"]), d["n"])
    s = th.tensor(sm["score"], dtype=th.float32, device=DEV).reshape(-1, 1)
    got = S.edge_softmax(g, s).reshape(-1).cpu().numpy()
    np.testing.assert_allclose(got, np.array(sm["out"], np.float32), rtol=1e-6, equal_nan=True)
    ref = O.edge_softmax(O.RefGraph(np.array(sm["src"]), np.array(sm["dst"]), d["n"]),
                         np.array(sm["score"], np.float32).reshape(-1, 1)).reshape(-1)
    np.testing.assert_allclose(got, ref, rtol=1e-6, equal_nan=True)
