"""The reference's specialisation tests (tests/compute/test_specialization.py:9-400)
restated: the builtin message/reduce paths of update_all / send_and_recv / pull
(v2v, e2v, multiple functions at once, apply_node_func) on its 10-node graph,
with 1-D and 2-D node features and 1-D / (E, 1) edge weights.  The reference
checks each builtin path against the same computation written as Python UDFs
(mailbox reduce); UDF reduces are outside this engine's scope, so the UDF side
is restated as an fp64 torch computation over the edge list (same numbers),
compared at the reference's F.allclose tolerance (1e-4)."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
D = 5


def generate_graph(seed=0):
    """test_specialization.py:9-21: 0 -> 1..8 -> 9, back edge 9 -> 0 (17 edges)."""
    g = dgl.DGLGraph()
    g.add_nodes(10)
    for i in range(1, 9):
        g.add_edge(0, i)
        g.add_edge(i, 9)
    g.add_edge(9, 0)
    gen = th.Generator().manual_seed(seed)
    g.ndata["f1"] = th.randn(10, generator=gen).to(DEV)
    g.ndata["f2"] = th.randn(10, D, generator=gen).to(DEV)
    w = th.randn(17, generator=gen).to(DEV)
    g.edata["e1"] = w
    g.edata["e2"] = w.unsqueeze(1)
    return g


def _edges(g):
    s, d, e = g._graph.edges()
    return th.as_tensor(s), th.as_tensor(d), th.as_tensor(e)


def _udf_sum(g, feat, eids, weight=None):
    """mailbox sum of src feature (times edge weight) over the given edges, fp64."""
    s, d, _ = _edges(g)
    eids = th.as_tensor(eids, dtype=th.long)
    x = feat.detach().double().cpu()
    msg = x[s[eids]]
    if weight is not None:
        w = weight.detach().double().cpu()[eids]
        msg = msg * (w if msg.dim() == w.dim() else w.reshape((-1,) + (1,) * (msg.dim() - 1)))
    out = th.zeros_like(x)
    out.index_add_(0, d[eids], msg)
    return out, th.unique(d[eids])


def _close(a, b):
    assert th.allclose(a.detach().double().cpu(), b, rtol=1e-4, atol=1e-4), (a, b)


def _apply(nodes):
    return {k: 2 * v for k, v in nodes.data.items() if k in ("f1", "f2")}


@pytest.mark.parametrize("fld", ["f1", "f2"])
def test_v2v_update_all(fld):
    g = generate_graph()
    v1 = g.ndata[fld].clone()
    g.update_all(fn.copy_src(src=fld, out="m"), fn.sum(msg="m", out=fld),
                 lambda nodes: {fld: 2 * nodes.data[fld]})
    ref, _ = _udf_sum(g, v1, np.arange(17))
    _close(g.ndata[fld], 2 * ref)
    g.ndata[fld] = v1
    w = "e1" if fld == "f1" else "e2"
    g.update_all(fn.src_mul_edge(src=fld, edge=w, out="m"), fn.sum(msg="m", out=fld),
                 lambda nodes: {fld: 2 * nodes.data[fld]})
    ref, _ = _udf_sum(g, v1, np.arange(17), g.edata["e1"])
    _close(g.ndata[fld], 2 * ref)


@pytest.mark.parametrize("fld", ["f1", "f2"])
@pytest.mark.parametrize("mode", ["snr", "pull"])
def test_v2v_partial(fld, mode):
    """send_and_recv on (u, v) pairs (test_v2v_snr) and pull on nodes
    (test_v2v_pull): receivers get reduce + apply, other nodes keep their value."""
    g = generate_graph()
    s, d, _ = _edges(g)
    if mode == "snr":
        u, v = [0, 0, 0, 3, 4, 9], [1, 2, 3, 9, 9, 0]
        eids = [int(((s == a) & (d == b)).nonzero()[0]) for a, b in zip(u, v)]
    else:
        nodes = [1, 2, 3, 9]
        eids = [int(e) for e in range(17) if int(d[e]) in nodes]
    for weighted in (False, True):
        v1 = g.ndata[fld].clone()
        w = "e1" if fld == "f1" else "e2"
        mfunc = fn.src_mul_edge(src=fld, edge=w, out="m") if weighted else fn.copy_src(src=fld, out="m")
        rfunc = fn.sum(msg="m", out=fld)
        afunc = lambda nb: {fld: 2 * nb.data[fld]}  # noqa: E731
        if mode == "snr":
            g.send_and_recv((u, v), mfunc, rfunc, afunc)
        else:
            g.pull(nodes, mfunc, rfunc, afunc)
        ref, recv = _udf_sum(g, v1, eids, g.edata["e1"] if weighted else None)
        want = v1.detach().double().cpu().clone()
        want[recv] = 2 * ref[recv]
        _close(g.ndata[fld], want)
        g.ndata[fld] = v1


def test_v2v_update_all_multi_fn():
    """test_specialization.py:145-182: one message to two reducers, two messages
    to three reducers (the same field reduced twice)."""
    g = generate_graph()
    fld = "f2"
    g.update_all(fn.copy_src(src=fld, out="m"), [fn.sum(msg="m", out="v2"), fn.sum(msg="m", out="v3")])
    ref, _ = _udf_sum(g, g.ndata[fld], np.arange(17))
    _close(g.ndata["v2"], ref)
    _close(g.ndata["v3"], ref)
    g.update_all([fn.src_mul_edge(src=fld, edge="e1", out="m1"),
                  fn.src_mul_edge(src=fld, edge="e2", out="m2")],
                 [fn.sum(msg="m1", out="v1"), fn.sum(msg="m2", out="v2"),
                  fn.sum(msg="m1", out="v3")])
    ref, _ = _udf_sum(g, g.ndata[fld], np.arange(17), g.edata["e1"])
    for k in ("v1", "v2", "v3"):
        _close(g.ndata[k], ref)


@pytest.mark.parametrize("mode", ["update_all", "snr", "recv"])
def test_e2v_multi_fn(mode):
    """test_specialization.py:232-345: edge features reduced to nodes (copy_edge)
    with two reducers at once and an apply function."""
    g = generate_graph()
    gen = th.Generator().manual_seed(5)
    g.edata["m1"] = th.randn(17, D, generator=gen).to(DEV)
    g.edata["m2"] = th.randn(17, D, generator=gen).to(DEV)
    s, d, _ = _edges(g)
    old = g.ndata["f2"].clone()
    r = [fn.sum(msg="a", out="r1"), fn.sum(msg="b", out="r2")]
    m = [fn.copy_edge(edge="m1", out="a"), fn.copy_edge(edge="m2", out="b")]
    if mode == "update_all":
        eids = list(range(17))
        g.update_all(m, r, lambda nb: {"f2": nb.data["r1"] + nb.data["r2"]})
    elif mode == "snr":
        u, v = [0, 0, 0, 3, 4, 9], [1, 2, 3, 9, 9, 0]
        eids = [int(((s == a) & (d == b)).nonzero()[0]) for a, b in zip(u, v)]
        g.send_and_recv((u, v), m, r, lambda nb: {"f2": nb.data["r1"] + nb.data["r2"]})
    else:  # pull on the receivers = recv after send on those edges
        nodes = [1, 2, 3, 9]
        eids = [int(e) for e in range(17) if int(d[e]) in nodes]
        g.pull(nodes, m, r, lambda nb: {"f2": nb.data["r1"] + nb.data["r2"]})
    e = th.as_tensor(eids)
    r1 = th.zeros(10, D, dtype=th.float64).index_add_(0, d[e], g.edata["m1"].double().cpu()[e])
    r2 = th.zeros(10, D, dtype=th.float64).index_add_(0, d[e], g.edata["m2"].double().cpu()[e])
    recv = th.unique(d[e])
    want = old.double().cpu().clone()
    want[recv] = (r1 + r2)[recv]
    _close(g.ndata["f2"], want)


def test_update_all_multi_fallback():
    """test_specialization.py:347-400: two weighted messages (1-D and (E, 1)
    weights) on a D-dim field, two reducers at once == one at a time."""
    g = generate_graph()
    gen = th.Generator().manual_seed(7)
    g.ndata["h"] = th.randn(10, D, generator=gen).to(DEV)
    g.edata["w1"] = th.randn(17, generator=gen).to(DEV)
    g.edata["w2"] = th.randn(17, D, generator=gen).to(DEV)
    g.update_all(fn.src_mul_edge(src="h", edge="w1", out="m1"), fn.sum(msg="m1", out="o1"))
    o1 = g.ndata.pop("o1")
    g.update_all(fn.src_mul_edge(src="h", edge="w2", out="m2"), fn.sum(msg="m2", out="o2"))
    o2 = g.ndata.pop("o2")
    ref1, _ = _udf_sum(g, g.ndata["h"], np.arange(17), g.edata["w1"])
    ref2, _ = _udf_sum(g, g.ndata["h"], np.arange(17), g.edata["w2"])
    _close(o1, ref1)
    _close(o2, ref2)
    g.update_all([fn.src_mul_edge(src="h", edge="w1", out="m1"),
                  fn.src_mul_edge(src="h", edge="w2", out="m2")],
                 [fn.sum(msg="m1", out="o1"), fn.sum(msg="m2", out="o2")])
    _close(g.ndata["o1"], ref1)
    _close(g.ndata["o2"], ref2)
