"""The row-owned edge softmax (kernels_softmax.hip k_sm_owned / k_sm_hub), taken when
the in-CSR's edge ids are its positions (a position view, a destination-sorted graph):
forward and backward against an fp64 softmax per destination and against the chunked
row pass + edge pass (DGLMI_SOFTMAX_OWNED=0), on degree sequences that put row ends on
every boundary the walk has -- a step (L positions), a window (W), the hub threshold
(T = 2W) -- plus rows of 0-3 edges (several rows inside one step), hub rows many windows
long, and masked / NaN / +inf logits.  Reference: python/dgl/nn/pytorch/softmax.py:33-114."""
import numpy as np
import pytest
import torch as th

import dgl
from dgl import kernel as K

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _shape(H):
    """(step, window, hub threshold) of the walk H takes: four values per lane for H <= 4
    (QuadWalk: 4 / H positions per lane, 64 * 4 / H a step), else V = 4 heads of one
    position per lane.  Windows are 2048 positions either way."""
    V = min(H, 4)
    L = 64 * 4 // H if H <= 2 else 64 // (H // V)
    W = 2048
    return L, W, 2 * W


def _degrees(H, seed):
    L, W, T = _shape(H)
    rs = np.random.RandomState(seed)
    edge = [0, 1, 2, 3, 4, 5, 63, 64, 65, L - 1, L, L + 1, W - 1, W, W + 1, T - 1, T, T + 1,
            3 * W + 5, 11 * W + 3]
    tiny = list(rs.randint(0, 4, 3000))
    mid = list(rs.randint(1, 3 * L, 400))
    big = list(rs.randint(W // 2, T + 1, 60))
    deg = edge + tiny + mid + big + edge[::-1]
    rs.shuffle(deg)
    return np.array(deg, dtype=np.int64)


def _graph(deg, seed):
    n = len(deg)
    rs = np.random.RandomState(seed)
    dst = np.repeat(np.arange(n), deg)
    src = rs.randint(0, n, len(dst))
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    return g._graph.get_immutable_gidx(DEV)


def _fp64(rows, s, n):
    s64 = s.double()
    mx = th.full((n,) + s.shape[1:], -float("inf"), dtype=th.float64, device=DEV)
    mx = mx.index_reduce(0, rows, s64, "amax")
    ex = th.exp(s64 - mx[rows])
    den = th.zeros_like(mx).index_add_(0, rows, ex)
    return ex / den[rows]


@pytest.mark.parametrize("H", [1, 2, 4, 8, 16])
def test_owned_softmax_fp64_and_chunked(H, monkeypatch):
    deg = _degrees(H, H)
    gidx = _graph(deg, H + 1)
    view = gidx.position_view("in")
    m = int(deg.sum())
    rows = view.in_csr.rows.long()
    gen = th.Generator(device=DEV).manual_seed(H)
    s = th.randn(m, H, device=DEV, generator=gen) * 3
    ga = th.randn(m, H, device=DEV, generator=gen)
    res = {}
    for owned in ("1", "0"):
        monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
        out, gs = th.empty_like(s), th.empty_like(s)
        K.edge_softmax_forward(view, s, out)
        K.edge_softmax_backward(view, out, ga, gs)
        res[owned] = (out, gs)
    (a1, g1), (a0, g0) = res["1"], res["0"]
    ref = _fp64(rows, s, len(deg))
    assert th.allclose(a1.double(), ref, rtol=1e-5, atol=1e-7)
    assert th.allclose(a1, a0, rtol=1e-5, atol=1e-7)
    # backward: a ga - a sum(a ga), fp64 from the fp32 forward output
    a64, g64 = a1.double(), ga.double()
    S = th.zeros((len(deg), H), dtype=th.float64, device=DEV).index_add_(0, rows, a64 * g64)
    gref = a64 * g64 - a64 * S[rows]
    assert th.allclose(g1.double(), gref, rtol=1e-4, atol=1e-6)
    assert th.allclose(g1, g0, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("mode", ["stored", "leaky", "node_logits"])
@pytest.mark.parametrize("H", [1, 2, 4])
def test_quad_walk_matches_plain_walk(H, mode, monkeypatch):
    """H <= 4 on the row-owned walk: four values per lane (QuadWalk, 16-B loads, rows that
    start and end inside one lane's positions finished by that lane) against one position
    per lane (DGLMI_SOFTMAX_QUAD=0) and fp64 -- stored logits, the fused leaky_relu and
    the node logits, forward and backward, on degree sequences that end rows inside a
    lane's positions, on step, window and hub boundaries."""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "1")
    deg = _degrees(H, 80 + H)
    n = len(deg)
    gidx = _graph(deg, 81 + H)
    view = gidx.position_view("in")
    rows = view.in_csr.rows.long()
    m = int(deg.sum())
    gen = th.Generator(device=DEV).manual_seed(H + 11)
    el = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    er = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    s = th.randn(m, H, 1, device=DEV, generator=gen) * 3
    ga = th.randn(m, H, 1, device=DEV, generator=gen)
    slope = 0.2
    res = {}
    for quad in ("1", "0"):
        monkeypatch.setenv("DGLMI_SOFTMAX_QUAD", quad)
        a, gs = th.empty_like(s), th.empty_like(s)
        if mode == "stored":
            K.edge_softmax_forward(view, s, a)
            K.edge_softmax_backward(view, a, ga, gs)
        elif mode == "leaky":
            K.edge_softmax_leaky_forward(view, s, slope, a)
            K.edge_softmax_leaky_backward(view, a, ga, s, slope, gs)
        else:
            K.edge_softmax_node_logits_forward(view, el, er, slope, a)
            K.edge_softmax_node_logits_backward(view, a, ga, el, er, slope, gs)
        res[quad] = (a, gs)
    (a1, g1), (a0, g0) = res["1"], res["0"]
    assert th.allclose(a1, a0, rtol=1e-5, atol=1e-7)
    assert th.allclose(g1, g0, rtol=1e-4, atol=1e-6)
    pre = s if mode != "node_logits" else el[view.in_csr.indices.long()] + er[rows]
    pre = pre.reshape(m, H)
    x = pre if mode == "stored" else th.nn.functional.leaky_relu(pre, slope)
    ref = _fp64(rows, x, n)
    assert th.allclose(a1.reshape(m, H).double(), ref, rtol=1e-5, atol=1e-7)
    a64, g64 = a1.reshape(m, H).double(), ga.reshape(m, H).double()
    S = th.zeros((n, H), dtype=th.float64, device=DEV).index_add_(0, rows, a64 * g64)
    gref = a64 * g64 - a64 * S[rows]
    if mode != "stored":
        gref = th.where(pre > 0, gref, gref * slope)
    assert th.allclose(g1.reshape(m, H).double(), gref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("mode", ["stored", "leaky", "node_logits"])
@pytest.mark.parametrize("H", [1, 2])
def test_quad_edge_pass_bit_identical(H, mode, monkeypatch):
    """The edge pass in edge-id order (a graph whose edges are not sorted by destination)
    with 4 / H edges per lane (k_sm_edges_q) and with the rows' statistics packed side by
    side (k_sm_pack; DGLMI_SOFTMAX_PACK=0: the two arrays) gives the one-edge-per-lane,
    two-array pass's bits,
    forward and backward, for stored logits, the fused leaky_relu and the node logits --
    on an edge count that is not a multiple of 4 (the last lane's partial quad) -- and
    matches fp64."""
    deg = _degrees(H, 90 + H)
    deg[0] += 3 - int(deg.sum()) % 4  # nnz = 3 (mod 4)
    n = len(deg)
    rs = np.random.RandomState(91 + H)
    dst = np.repeat(np.arange(n), deg)
    src = rs.randint(0, n, len(dst))
    perm = rs.permutation(len(dst))
    gg = dgl.DGLGraph()
    gg.add_nodes(n)
    gg.add_edges(src[perm], dst[perm])
    g = gg._graph.get_immutable_gidx(DEV)
    assert not (g.eid_identity_bits() & 1)
    m = len(dst)
    assert m % 4 == 3
    gen = th.Generator(device=DEV).manual_seed(H + 13)
    el = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    er = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    s = th.randn(m, H, 1, device=DEV, generator=gen) * 3
    s[7, 0, 0] = -float("inf")
    s[m - 1, 0, 0] = float("nan")
    ga = th.randn(m, H, 1, device=DEV, generator=gen)
    res = {}
    for quad, pack in (("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")):
        monkeypatch.setenv("DGLMI_SOFTMAX_QUAD", quad)
        monkeypatch.setenv("DGLMI_SOFTMAX_PACK", pack)
        a, gs = th.empty_like(s), th.empty_like(s)
        if mode == "stored":
            K.edge_softmax_forward(g, s, a)
            K.edge_softmax_backward(g, a, ga, gs)
        elif mode == "leaky":
            K.edge_softmax_leaky_forward(g, s, 0.2, a)
            K.edge_softmax_leaky_backward(g, a, ga, s, 0.2, gs)
        else:
            K.edge_softmax_node_logits_forward(g, el, er, 0.2, a)
            K.edge_softmax_node_logits_backward(g, a, ga, el, er, 0.2, gs)
        res[quad + pack] = (a, gs)
    for key in ("01", "10", "00"):  # every form gives the same bits
        for x, y in zip(res["11"], res[key]):
            assert th.equal(th.isnan(x), th.isnan(y)) and th.equal(x[~th.isnan(y)], y[~th.isnan(y)])
    rows = th.from_numpy(dst[perm]).to(DEV)
    pre = s.reshape(m, H) if mode != "node_logits" else (el[th.from_numpy(src[perm]).to(DEV)] + er[rows]).reshape(m, H)
    x = pre if mode == "stored" else th.nn.functional.leaky_relu(pre, 0.2)
    ref = _fp64(rows, x, n)
    a1 = res["11"][0].reshape(m, H)
    fin = ~th.isnan(ref)
    assert th.equal(th.isnan(a1), ~fin)
    assert th.allclose(a1[fin].double(), ref[fin], rtol=1e-5, atol=1e-7)


def test_owned_softmax_deterministic(monkeypatch):
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "1")
    deg = _degrees(8, 3)
    view = _graph(deg, 4).position_view("in")
    s = th.randn(int(deg.sum()), 8, device=DEV)
    a = th.empty_like(s)
    b = th.empty_like(s)
    K.edge_softmax_forward(view, s, a)
    K.edge_softmax_forward(view, s, b)
    assert th.equal(a, b)


@pytest.mark.parametrize("H", [1, 8])
def test_owned_softmax_special_values(H, monkeypatch):
    """-inf logits get 0, an all -inf row NaN, a +inf or NaN logit makes its row NaN
    (exp(s - max) / sum, as the decomposition) -- in short rows, in rows cut by steps
    and in hub rows cut into pieces."""
    L, W, T = _shape(H)
    deg = np.array([3, L + 2, 2, 5, W + 7, T + 9, 4, 3 * W, 1, 6, T + 5, 3, L * 3], dtype=np.int64)
    view = _graph(deg, 7).position_view("in")
    rows = view.in_csr.rows.long()
    m = int(deg.sum())
    s = th.randn(m, H, device=DEV)
    starts = np.concatenate([[0], np.cumsum(deg)[:-1]])
    s[int(starts[0]) + 1, 0] = -float("inf")          # one masked logit
    s[int(starts[2]):int(starts[2]) + 2] = -float("inf")  # an all-masked row
    s[int(starts[3]) + 4, 0] = float("nan")           # NaN in a short row
    s[int(starts[4]) + W, 0] = float("inf")           # +inf in a row cut by a window
    s[int(starts[5]) + 2 * W + 3, 0] = -float("inf")   # masked inside a hub row
    s[int(starts[7]) + W + 1, 0] = float("nan")       # NaN in a hub row
    # rows masked everywhere but one NaN (a NaN met while the running maximum is -inf):
    # a hub row, a short row, a row a few steps long
    for r, k in ((10, 2 * W + 17), (11, 1), (12, 2 * L + 5)):
        s[int(starts[r]):int(starts[r]) + int(deg[r])] = -float("inf")
        s[int(starts[r]) + k, 0] = float("nan")
    out = {}
    for owned in ("1", "0"):
        monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
        o = th.empty_like(s)
        K.edge_softmax_forward(view, s, o)
        out[owned] = o
    a, b = out["1"], out["0"]
    assert th.equal(th.isnan(a), th.isnan(b))
    fin = ~th.isnan(b)
    assert th.allclose(a[fin], b[fin], rtol=1e-5, atol=1e-7)
    assert a[int(starts[0]) + 1, 0].item() == 0.0
    assert bool(th.isnan(a[int(starts[2]):int(starts[2]) + 2]).all())
    for r in (10, 11, 12):
        assert bool(th.isnan(a[int(starts[r]):int(starts[r]) + int(deg[r]), 0]).all())
    ref = _fp64(rows, s, len(deg))
    assert th.equal(th.isnan(a), th.isnan(ref))
    assert th.allclose(a[fin].double(), ref[fin], rtol=1e-5, atol=1e-7)


def test_dst_sorted_graph_takes_owned_route(monkeypatch):
    """A whole graph whose edges came sorted by destination (in-CSR edge ids = positions)
    runs the row-owned walk through nn.edge_softmax, with the same values as the
    chunked route."""
    from dgl.nn.pytorch import edge_softmax
    from graphs import powerlaw
    src, dst, n = powerlaw(20_000, 400_000, seed=31)
    order = np.lexsort((src, dst))
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src[order], dst[order])
    assert g._graph.get_immutable_gidx(DEV).eid_identity_bits() & 1
    s = th.randn(len(src), 4, 1, device=DEV)
    res = {}
    for owned in ("1", "0"):
        monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", owned)
        x = s.clone().requires_grad_()
        a = edge_softmax(g, x)
        a.backward(th.ones_like(a) * th.arange(a.shape[0], device=DEV).reshape(-1, 1, 1) % 7)
        res[owned] = (a.detach(), x.grad)
    assert th.allclose(res["1"][0], res["0"][0], rtol=1e-5, atol=1e-7)
    assert th.allclose(res["1"][1], res["0"][1], rtol=1e-4, atol=1e-6)


def test_owned_softmax_64bit_offsets_bit_identical(monkeypatch):
    """The row-owned walk on a graph in the 64-bit layout (int64 offsets: IdxPtr wide)
    gives the 32-bit layout's bits, hub rows included."""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "1")
    deg = _degrees(8, 5)
    n = len(deg)
    rs = np.random.RandomState(6)
    dst = np.repeat(np.arange(n), deg)
    src = rs.randint(0, n, len(dst))
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    g64 = dgl.DGLGraph(g._graph.asbits(64))
    s = th.randn(len(dst), 8, device=DEV)
    ga = th.randn(len(dst), 8, device=DEV)
    res = []
    for gg in (g, g64):
        view = gg._graph.get_immutable_gidx(DEV).position_view("in")
        out, gs = th.empty_like(s), th.empty_like(s)
        K.edge_softmax_forward(view, s, out)
        K.edge_softmax_backward(view, out, ga, gs)
        res.append((out, gs))
    assert g64._graph.get_immutable_gidx(DEV).num_bits == 64
    assert th.equal(res[0][0], res[1][0]) and th.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("route", ["view_owned", "view_chunked", "graph"])
@pytest.mark.parametrize("H", [1, 2, 4, 8, 16])
def test_leaky_softmax_bit_identical(route, H, monkeypatch):
    """DGLMIEdgeSoftmaxLeakyForward / Backward (leaky_relu inside the softmax's passes)
    against torch's leaky_relu + the plain softmax entries on the same route: the same
    bits forward and backward, masked / NaN / +inf / zero logits included."""
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "0" if route == "view_chunked" else "1")
    deg = _degrees(H, 40 + H)
    if route == "graph":  # edges in shuffled order: the edge-id walk (chunked row pass)
        n = len(deg)
        rs = np.random.RandomState(41 + H)
        dst = np.repeat(np.arange(n), deg)
        src = rs.randint(0, n, len(dst))
        perm = rs.permutation(len(dst))
        gg = dgl.DGLGraph()
        gg.add_nodes(n)
        gg.add_edges(src[perm], dst[perm])
        g = gg._graph.get_immutable_gidx(DEV)
        assert not (g.eid_identity_bits() & 1)
    else:
        g = _graph(deg, 41 + H).position_view("in")
    m = int(deg.sum())
    gen = th.Generator(device=DEV).manual_seed(H + 7)
    x = th.randn(m, H, device=DEV, generator=gen) * 3
    x[5, 0] = -float("inf")
    x[17, 0] = 0.0
    x[m // 2, 0] = float("nan")
    x[m // 3, 0] = float("inf")
    ga = th.randn(m, H, device=DEV, generator=gen)
    slope = 0.2
    a1, g1 = th.empty_like(x), th.empty_like(x)
    K.edge_softmax_leaky_forward(g, x, slope, a1)
    K.edge_softmax_leaky_backward(g, a1, ga, x, slope, g1)
    y = th.nn.functional.leaky_relu(x, slope)
    a0, gy = th.empty_like(x), th.empty_like(x)
    K.edge_softmax_forward(g, y, a0)
    K.edge_softmax_backward(g, a0, ga, gy)
    g0 = th.ops.aten.leaky_relu_backward(gy, x, slope, False)
    assert th.equal(th.isnan(a1), th.isnan(a0)) and th.equal(a1[~th.isnan(a0)], a0[~th.isnan(a0)])
    assert th.equal(th.isnan(g1), th.isnan(g0)) and th.equal(g1[~th.isnan(g0)], g0[~th.isnan(g0)])


@pytest.mark.parametrize("route", ["view_owned", "view_chunked", "graph"])
@pytest.mark.parametrize("H", [1, 2, 4, 8, 16])
def test_node_logit_softmax_bit_identical(route, H, monkeypatch):
    """DGLMIEdgeSoftmaxNodeLogits{Forward,Backward} (the logit el[u] + er[v] computed
    where the softmax reads it) against the stored-logit chain on the same route -- the
    u_add_v SDDMM, then the leaky softmax entries: the same bits forward and backward,
    masked / NaN / +inf node logits included; the edge-id-order pass (graph route) reads
    the sources from the COO."""
    from dgl import backend as B
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "0" if route == "view_chunked" else "1")
    deg = _degrees(H, 60 + H)
    n = len(deg)
    rs = np.random.RandomState(61 + H)
    dst = np.repeat(np.arange(n), deg)
    src = rs.randint(0, n, len(dst))
    gg = dgl.DGLGraph()
    gg.add_nodes(n)
    if route == "graph":
        perm = rs.permutation(len(dst))
        gg.add_edges(src[perm], dst[perm])
        g = gg._graph.get_immutable_gidx(DEV)
        assert not (g.eid_identity_bits() & 1)
    else:
        gg.add_edges(src, dst)
        g = gg._graph.get_immutable_gidx(DEV).position_view("in")
    m = int(deg.sum())
    gen = th.Generator(device=DEV).manual_seed(H + 9)
    el = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    er = th.randn(n, H, 1, device=DEV, generator=gen) * 2
    el[3, 0, 0] = -float("inf")
    er[7, 0, 0] = float("nan")
    el[11, 0, 0] = float("inf")
    ga = th.randn(m, H, 1, device=DEV, generator=gen)
    slope = 0.2
    a1, g1 = th.empty(m, H, 1, device=DEV), th.empty(m, H, 1, device=DEV)
    K.edge_softmax_node_logits_forward(g, el, er, slope, a1)
    K.edge_softmax_node_logits_backward(g, a1, ga, el, er, slope, g1)
    e = th.empty(m, H, 1, device=DEV)
    K.binary_op_reduce("none", "add", g, B.SRC, B.DST, el, er, e)
    a0, g0 = th.empty_like(e), th.empty_like(e)
    K.edge_softmax_leaky_forward(g, e, slope, a0)
    K.edge_softmax_leaky_backward(g, a0, ga, e, slope, g0)
    for x, y in ((a1, a0), (g1, g0)):
        assert th.equal(th.isnan(x), th.isnan(y)) and th.equal(x[~th.isnan(y)], y[~th.isnan(y)])


def test_node_logit_softmax_64bit_and_empty():
    """The node-logit entries on a graph in the 64-bit layout give the 32-bit layout's
    bits (position view, hub rows included), and on an edgeless graph they return
    without touching their outputs."""
    deg = _degrees(8, 70)
    n = len(deg)
    rs = np.random.RandomState(71)
    dst = np.repeat(np.arange(n), deg)
    src = rs.randint(0, n, len(dst))
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    g64 = dgl.DGLGraph(g._graph.asbits(64))
    el = th.randn(n, 8, 1, device=DEV)
    er = th.randn(n, 8, 1, device=DEV)
    ga = th.randn(len(dst), 8, 1, device=DEV)
    res = []
    for gg in (g, g64):
        view = gg._graph.get_immutable_gidx(DEV).position_view("in")
        a, gs = th.empty_like(ga), th.empty_like(ga)
        K.edge_softmax_node_logits_forward(view, el, er, 0.2, a)
        K.edge_softmax_node_logits_backward(view, a, ga, el, er, 0.2, gs)
        res.append((a, gs))
    assert g64._graph.get_immutable_gidx(DEV).num_bits == 64
    assert th.equal(res[0][0], res[1][0]) and th.equal(res[0][1], res[1][1])
    e0 = dgl.DGLGraph()
    e0.add_nodes(5)
    gi = e0._graph.get_immutable_gidx(DEV)
    out = th.full((0, 8, 1), 7.0, device=DEV)
    K.edge_softmax_node_logits_forward(gi, el[:5], er[:5], 0.2, out)
    K.edge_softmax_node_logits_backward(gi, out, out, el[:5], er[:5], 0.2, out)
