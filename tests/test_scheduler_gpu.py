"""The reference's own scheduler tests, restated on the device: message-passing
entry points, degree bucketing (mailbox shapes), zero-in-degree handling through
the frame initializers, the pending-message indicator of send / recv, and
in-place writes.

Sources (python/dgl semantics these pin):
* tests/compute/test_basics.py:49-614  (update routines, 0-degree nodes, multigraph sends)
* tests/compute/test_multi_send_recv.py:43-340
* tests/compute/test_inplace_update.py:25-296
Reference features are ``F.randn`` draws; here the same shapes, seeded per test
(tests/conftest.py).  Builtin message / reduce pairs run the HIP kernels; UDF
reducers run the device degree bucketing (graph.py)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch as th

import dgl
import dgl.function as fn
from dgl import DGLGraph
from dgl._ffi import DGLError

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
D = 5
SHAPES = set()


def randn(*shape):
    return th.randn(*shape, device=DEV)


def allclose(a, b):
    a, b = th.as_tensor(a), th.as_tensor(b)
    return th.allclose(a.cpu().double(), b.cpu().double(), rtol=1e-4, atol=1e-4)


def message_func(edges):
    assert edges.src["h"].dim() == 2 and edges.src["h"].shape[1] == D
    return {"m": edges.src["h"]}


def reduce_func(nodes):
    msgs = nodes.mailbox["m"]
    SHAPES.add(tuple(msgs.shape))
    assert msgs.dim() == 3 and msgs.shape[2] == D
    return {"accum": msgs.sum(1)}


def apply_node_func(nodes):
    return {"h": nodes.data["h"] + nodes.data["accum"]}


def init2(shape, dtype, ctx, ids):
    return 2 + th.zeros(shape, dtype=dtype, device=ctx)


def generate_graph(back_edge=True):
    """test_basics.py:27-47: 0 -> 1..8 -> 9 (-> 0)."""
    g = DGLGraph()
    g.add_nodes(10)
    for i in range(1, 9):
        g.add_edge(0, i)
        g.add_edge(i, 9)
    if back_edge:
        g.add_edge(9, 0)
    g.ndata["h"] = randn(10, D)
    g.edata["w"] = randn(g.number_of_edges(), D)
    g.set_n_initializer(dgl.init.zero_initializer)
    g.set_e_initializer(dgl.init.zero_initializer)
    return g


# ---- test_basics.py ------------------------------------------------------------
def test_batch_send():
    g = generate_graph()

    def _fmsg(edges):
        assert tuple(edges.src["h"].shape) == (5, D)
        return {"m": edges.src["h"]}
    g.register_message_func(_fmsg)
    g.send((th.tensor([0, 0, 0, 0, 0]), th.tensor([1, 2, 3, 4, 5])))
    g.send((th.tensor([0]), th.tensor([1, 2, 3, 4, 5])))
    g.send((th.tensor([1, 2, 3, 4, 5]), th.tensor([9])))


def test_batch_recv():
    g = generate_graph()
    g.register_message_func(message_func)
    g.register_reduce_func(reduce_func)
    g.register_apply_node_func(apply_node_func)
    u = th.tensor([0, 0, 0, 4, 5, 6])
    v = th.tensor([1, 2, 3, 9, 9, 9])
    SHAPES.clear()
    g.send((u, v))
    g.recv(th.unique(v))
    assert SHAPES == {(1, 3, D), (3, 1, D)}


def test_apply_nodes_and_edges():
    g = generate_graph()
    g.register_apply_node_func(lambda nodes: {"h": nodes.data["h"] * 2})
    old = g.ndata["h"]
    g.apply_nodes()
    assert allclose(old * 2, g.ndata["h"])
    u = th.tensor([0, 3, 4, 6])
    g.apply_nodes(lambda nodes: {"h": nodes.data["h"] * 0.}, u)
    assert allclose(g.ndata["h"][u.to(DEV)], th.zeros(4, D))

    g.register_apply_edge_func(lambda edges: {"w": edges.data["w"] * 2})
    old = g.edata["w"]
    g.apply_edges()
    assert allclose(old * 2, g.edata["w"])
    u = th.tensor([0, 0, 0, 4, 5, 6])
    v = th.tensor([1, 2, 3, 9, 9, 9])
    g.apply_edges(lambda edges: {"w": edges.data["w"] * 0.}, (u, v))
    eid = g.edge_ids(u, v)
    assert allclose(g.edata["w"][eid.to(DEV)], th.zeros(6, D))


def test_update_routines():
    g = generate_graph()
    g.register_message_func(message_func)
    g.register_reduce_func(reduce_func)
    g.register_apply_node_func(apply_node_func)
    SHAPES.clear()
    u, v = [0, 0, 0, 4, 5, 6], [1, 2, 3, 9, 9, 9]
    g.send_and_recv((u, v))
    assert SHAPES == {(1, 3, D), (3, 1, D)}
    with pytest.raises(DGLError):
        g.send_and_recv([u, v])
    SHAPES.clear()
    g.pull(th.tensor([1, 2, 3, 9]))
    assert SHAPES == {(1, 8, D), (3, 1, D)}
    SHAPES.clear()
    g.push(th.tensor([0, 1, 2, 3]))
    assert SHAPES == {(1, 3, D), (8, 1, D)}
    SHAPES.clear()
    g.update_all()
    assert SHAPES == {(1, 8, D), (9, 1, D)}


def _zero_deg_udfs(field_in="h", field_out="h"):
    def _message(edges):
        return {"m": edges.src["h"]}

    def _reduce(nodes):
        return {field_out: nodes.data[field_in] + nodes.mailbox["m"].sum(1)}

    def _apply(nodes):
        return {field_out: nodes.data[field_out] * 2}
    return _message, _reduce, _apply


def test_recv_0deg():
    g = DGLGraph()
    g.add_nodes(2)
    g.add_edge(0, 1)
    m, r, a = _zero_deg_udfs()
    g.register_message_func(m)
    g.register_reduce_func(r)
    g.register_apply_node_func(a)
    g.set_n_initializer(init2, "h")
    old = randn(2, 5)
    g.ndata["h"] = old
    g.send((0, 1))
    g.recv([0, 1])
    new = g.ndata.pop("h")
    assert allclose(new[0], th.full((5,), 4.))        # initializer, then apply
    assert allclose(new[1], old.sum(0) * 2)
    old = randn(2, 5)
    g.ndata["h"] = old
    g.send((0, 1))
    g.recv(0)                                          # only a 0-degree node: = apply
    new = g.ndata.pop("h")
    assert allclose(new[0], 2 * old[0])
    assert allclose(new[1], old[1])


def test_recv_0deg_newfld():
    g = DGLGraph()
    g.add_nodes(2)
    g.add_edge(0, 1)
    m, r, a = _zero_deg_udfs("h", "h1")
    g.register_message_func(m)
    g.register_reduce_func(r)
    g.register_apply_node_func(a)
    old = randn(2, 5)
    g.set_n_initializer(init2, "h1")
    g.ndata["h"] = old
    g.send((0, 1))
    g.recv([0, 1])
    new = g.ndata.pop("h1")
    assert allclose(new[0], th.full((5,), 4.))
    assert allclose(new[1], old.sum(0) * 2)
    old = randn(2, 5)
    g.ndata["h"] = old
    g.ndata["h1"] = th.full((2, 5), -1, dtype=th.int64, device=DEV)
    g.send((0, 1))
    g.recv(0)
    new = g.ndata.pop("h1")
    assert th.equal(new[0].cpu(), th.full((5,), -2, dtype=th.int64))
    assert th.equal(new[1].cpu(), th.full((5,), -1, dtype=th.int64))


def test_update_all_0deg():
    g = DGLGraph()
    g.add_nodes(5)
    for s in (1, 2, 3, 4):
        g.add_edge(s, 0)
    m, r, a = _zero_deg_udfs()
    g.set_n_initializer(init2, "h")
    old = randn(5, 5)
    g.ndata["h"] = old
    g.update_all(m, r, a)
    new = g.ndata["h"]
    assert allclose(new[1:], 2 * (2 + th.zeros(4, 5)))
    assert allclose(new[0], 2 * old.sum(0))
    g = DGLGraph()                                     # no edge at all: = apply
    g.add_nodes(5)
    g.set_n_initializer(init2, "h")
    g.ndata["h"] = old
    g.update_all(m, r, a)
    assert allclose(g.ndata["h"], 2 * old)


def test_update_all_0deg_builtin_keeps_no_field():
    """Edgeless graph with builtins: scheduler.py downgrades to apply, so the
    reduce output field is never created."""
    g = DGLGraph()
    g.add_nodes(4)
    g.ndata["h"] = randn(4, 3)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "s"))
    assert "s" not in g.ndata


def test_pull_0deg():
    g = DGLGraph()
    g.add_nodes(2)
    g.add_edge(0, 1)
    m, r, a = _zero_deg_udfs()
    g.register_message_func(m)
    g.register_reduce_func(r)
    g.register_apply_node_func(a)
    g.set_n_initializer(init2, "h")
    old = randn(2, 5)
    g.ndata["h"] = old
    g.pull([0, 1])
    new = g.ndata.pop("h")
    assert allclose(new[0], th.full((5,), 4.))
    assert allclose(new[1], old.sum(0) * 2)
    old = randn(2, 5)
    g.ndata["h"] = old
    g.pull(0)
    new = g.ndata.pop("h")
    assert allclose(new[0], 2 * old[0])
    assert allclose(new[1], old[1])


def test_send_multigraph():
    g = DGLGraph()
    g.add_nodes(3)
    for _ in range(3):
        g.add_edge(0, 1)
    g.add_edge(2, 1)

    def _message_a(edges):
        return {"a": edges.data["a"]}

    def _message_b(edges):
        return {"a": edges.data["a"] * 3}

    def _reduce(nodes):
        return {"a": nodes.mailbox["a"].max(1)[0]}

    def answer(*args):
        return th.stack(args, 0).max(0)[0]

    old = randn(4, 5)
    g.ndata["a"] = th.zeros(3, 5, device=DEV)
    g.edata["a"] = old
    g.send([0, 2], message_func=_message_a)
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], answer(old[0], old[2]))
    g.ndata["a"] = th.zeros(3, 5, device=DEV)
    g.send([0, 2, 3], message_func=_message_a)
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], answer(old[0], old[2], old[3]))
    g.ndata["a"] = th.zeros(3, 5, device=DEV)          # (u, v) pairs: every parallel edge
    g.send(([0, 2], [1, 1]), _message_a)
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], old.max(0)[0])
    g.ndata["a"] = th.zeros(3, 5, device=DEV)          # consecutive sends, one recv
    g.send((2, 1), _message_a)
    g.send([0, 1], message_func=_message_b)
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], answer(old[0] * 3, old[1] * 3, old[3]))
    g.ndata["a"] = th.zeros(3, 5, device=DEV)
    g.send(0, message_func=_message_a)
    g.send(1, message_func=_message_b)
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], answer(old[0], old[1] * 3))
    g.ndata["a"] = th.zeros(3, 5, device=DEV)
    g.send_and_recv([0, 2, 3], message_func=_message_a, reduce_func=_reduce)
    assert allclose(g.ndata["a"][1], answer(old[0], old[2], old[3]))
    assert allclose(g.ndata["a"][th.tensor([0, 2], device=DEV)], th.zeros(2, 5))


def test_dynamic_addition_frames():
    n, d = 3, 1
    g = DGLGraph()
    g.add_nodes(n)
    g.ndata.update({"h1": randn(n, d), "h2": randn(n, d)})
    g.add_nodes(3)
    assert g.ndata["h1"].shape[0] == g.ndata["h2"].shape[0] == n + 3
    g.add_edge(0, 1)
    g.add_edge(1, 0)
    g.edata.update({"h1": randn(2, d), "h2": randn(2, d)})
    g.add_edges([0, 2], [2, 0])
    g.edata["h1"] = randn(4, d)
    assert g.edata["h1"].shape[0] == g.edata["h2"].shape[0] == 4
    g.add_edge(1, 2)
    g.edges[4].data["h1"] = randn(1, d)
    assert g.edata["h1"].shape[0] == g.edata["h2"].shape[0] == 5
    g.add_edge(2, 1, {"h1": randn(1, d)})
    assert len(g.edata["h1"]) == len(g.edata["h2"])


# ---- test_multi_send_recv.py -----------------------------------------------------
def test_multi_send():
    g = generate_graph(back_edge=False)

    def _fmsg(edges):
        assert tuple(edges.src["h"].shape) == (5, D)
        return {"m": edges.src["h"]}
    g.register_message_func(_fmsg)
    g.send((th.tensor([0, 0, 0, 0, 0]), th.tensor([1, 2, 3, 4, 5])))
    g.send((th.tensor([0]), th.tensor([1, 2, 3, 4, 5])))
    g.send((th.tensor([1, 2, 3, 4, 5]), th.tensor([9])))
    expected = np.zeros(g.number_of_edges(), np.int64)
    eid = g.edge_ids([0, 0, 0, 0, 0, 1, 2, 3, 4, 5], [1, 2, 3, 4, 5, 9, 9, 9, 9, 9])
    expected[eid.numpy()] = 1
    assert np.array_equal(g._get_msg_index(), expected)


def test_multi_recv():
    g = generate_graph(back_edge=False)
    h = g.ndata["h"]
    g.register_message_func(message_func)
    g.register_reduce_func(reduce_func)
    g.register_apply_node_func(apply_node_func)
    expected = np.zeros(g.number_of_edges(), np.int64)
    for u, v in (([4, 5, 6], [9]), ([0], [1, 2, 3])):   # two rounds of send + recv
        g.send((u, v))
        eid = g.edge_ids(u, v).numpy()
        expected[eid] = 1
        assert np.array_equal(g._get_msg_index(), expected)
        g.recv(v)
        expected[eid] = 0
        assert np.array_equal(g._get_msg_index(), expected)
    h1 = g.ndata["h"]
    g.ndata["h"] = h                                      # one send, two recvs
    g.send(([0, 0, 0, 4, 5, 6], [1, 2, 3, 9, 9, 9]))
    expected[g.edge_ids([0, 0, 0, 4, 5, 6], [1, 2, 3, 9, 9, 9]).numpy()] = 1
    assert np.array_equal(g._get_msg_index(), expected)
    for u, v in (([4, 5, 6], [9]), ([0], [1, 2, 3])):
        g.recv(v)
        expected[g.edge_ids(u, v).numpy()] = 0
        assert np.array_equal(g._get_msg_index(), expected)
    assert allclose(h1, g.ndata["h"])


def test_multi_recv_0deg():
    g = DGLGraph()
    m, r, a = _zero_deg_udfs()
    g.register_message_func(m)
    g.register_reduce_func(r)
    g.register_apply_node_func(a)
    g.set_n_initializer(init2)
    g.add_nodes(2)
    g.add_edge(0, 1)
    old = randn(2, 5)
    g.ndata["h"] = old
    g.send((0, 1))
    g.recv([0, 1])
    new = g.ndata["h"]
    assert allclose(new[0], th.full((5,), 4.))
    assert allclose(new[1], old.sum(0) * 2)
    g.recv([0])                                           # zero-degree node again: apply
    assert allclose(g.nodes[0].data["h"], th.full((1, 5), 8.))
    g.recv([1])                                           # message already consumed: apply
    assert allclose(g.nodes[1].data["h"], (old.sum(0) * 4).unsqueeze(0))


def test_send_twice_different_shape_msg_field():
    g = generate_graph(back_edge=False)
    g.send(message_func=lambda edges: {"h": edges.src["h"]})
    g.send(message_func=lambda edges: {"h": th.cat((edges.src["h"], edges.data["w"]), 1)})

    g = DGLGraph()
    g.set_n_initializer(dgl.init.zero_initializer)
    g.add_nodes(3)
    g.add_edge(0, 1)
    g.add_edge(2, 1)

    def _reduce(nodes):
        return {"a": nodes.mailbox["a"].max(1)[0]}
    old = randn(3, 5)
    g.ndata["a"] = old
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((0, 1), lambda edges: {"a": edges.src["a"] * 3})
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], old[0] * 3)
    g.ndata["a"] = old
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((2, 1), lambda edges: {"a": edges.src["a"] * 3})
    g.recv(1, _reduce)
    assert allclose(g.ndata["a"][1], th.stack([old[0], old[2] * 3], 0).max(0)[0])

    g = DGLGraph()
    g.set_n_initializer(dgl.init.zero_initializer)
    g.add_nodes(2)
    g.add_edge(0, 1)
    old_a, old_b = randn(2, 5), randn(2, 5)
    g.set_n_repr({"a": old_a, "b": old_b})
    g.send((0, 1), lambda edges: {"a": edges.src["a"]})
    g.send((0, 1), lambda edges: {"b": edges.src["b"]})
    g.recv([1], lambda nodes: {"a": nodes.mailbox["a"].sum(1), "b": nodes.mailbox["b"].sum(1)})
    rep = g.get_n_repr()
    assert allclose(rep["a"][1], old_a[0])
    assert allclose(rep["b"][1], old_b[0])


def test_dynamic_addition_send_recv():
    n, d = 3, 1
    g = DGLGraph()

    def _message(edges):
        return {"m": edges.src["h1"] + edges.dst["h2"] + edges.data["h1"] + edges.data["h2"]}
    g.register_message_func(_message)
    g.register_reduce_func(lambda nodes: {"h": nodes.mailbox["m"].sum(1)})
    g.register_apply_node_func(lambda nodes: {"h": nodes.data["h"]})
    g.set_n_initializer(dgl.init.zero_initializer)
    g.set_e_initializer(dgl.init.zero_initializer)
    g.add_nodes(n)
    g.ndata.update({"h1": randn(n, d), "h2": randn(n, d)})
    g.add_nodes(3)
    g.add_edge(0, 1)
    g.add_edge(1, 0)
    g.edata.update({"h1": randn(2, d), "h2": randn(2, d)})
    g.send()
    assert np.array_equal(g._get_msg_index(), np.ones(g.number_of_edges(), np.int64))
    g.add_edges([0, 2], [2, 0], {"h1": randn(2, d)})
    g.send(([0, 2], [2, 0]))
    g.recv(0)
    g.add_edge(1, 2)
    g.edges[4].data["h1"] = randn(1, d)
    g.send((1, 2))
    g.recv([1, 2])
    h = g.ndata.pop("h")
    g.send()                                              # a complete round again
    g.recv()
    assert allclose(h, g.ndata["h"])


def test_recv_no_send_and_clear():
    g = generate_graph(back_edge=False)
    g.recv(1, reduce_func)
    g.clear()
    g.add_nodes(3)
    g.add_edges([0, 1], [1, 2])
    g.set_n_initializer(dgl.init.zero_initializer)
    g.ndata["h"] = randn(3, D)
    g.send((1, 2), message_func)
    assert np.array_equal(g._get_msg_index(), np.array([0, 1]))
    g.recv(2, reduce_func)
    assert np.array_equal(g._get_msg_index(), np.array([0, 0]))


def test_send_recv_after_conversion():
    """The scipy half of test_multi_send_recv.py:298-340 (networkx is not installed
    here): a graph rebuilt from a COO matrix of the same edges gives the same
    send / recv results."""
    g = generate_graph(back_edge=False)
    row, col = g.all_edges()
    n = g.number_of_nodes()
    a = sp.coo_matrix((np.arange(len(row)), (row.numpy(), col.numpy())), shape=(n, n))
    g2 = DGLGraph()
    g2.add_nodes(5)
    g2.add_edges([1, 2, 4], [2, 3, 0])
    g2.set_n_initializer(dgl.init.zero_initializer)
    g2.from_scipy_sparse_matrix(a)
    g2.ndata["h"] = g.ndata["h"]
    for gg in (g, g2):
        gg.send(message_func=message_func)
        gg.recv([0, 1, 3, 5], reduce_func=reduce_func, apply_node_func=apply_node_func)
        gg.recv([0, 2, 4, 8], reduce_func=reduce_func, apply_node_func=apply_node_func)
    assert allclose(g.ndata["h"], g2.ndata["h"])


# ---- test_inplace_update.py --------------------------------------------------------
def inplace_graph():
    g = DGLGraph()
    g.add_nodes(10)
    for i in range(1, 9):
        g.add_edge(0, i)
        g.add_edge(i, 9)
    g.add_edge(9, 0)
    g.ndata["f"] = randn(10, D)
    g.edata["e"] = randn(17, D)
    return g


U = th.tensor([0, 0, 0, 3, 4, 9])
V = th.tensor([1, 2, 3, 9, 9, 0])


def _sum_f(nodes):
    return {"f": nodes.mailbox["m"].sum(1)}


def _apply2(nodes):
    return {"f": 2 * nodes.data["f"]}


@pytest.mark.parametrize("apply_func", [_apply2, None])
def test_inplace_recv(apply_func):
    g = inplace_graph()
    f = g.ndata["f"]
    msg = lambda edges: {"m": edges.src["f"] + edges.dst["f"]}  # noqa: E731
    g.send((U, V), msg)
    g.recv([0, 1, 2, 3, 9], _sum_f, apply_func)
    result = g.get_n_repr()["f"]
    for red in (_sum_f, fn.sum(msg="m", out="f")):        # degree bucketing, then e2v kernel
        v1 = f.clone()
        g.ndata["f"] = v1
        g.send((U, V), msg)
        g.recv([0, 1, 2, 3, 9], red, apply_func, inplace=True)
        r1 = g.get_n_repr()["f"]
        assert allclose(r1, result)
        assert allclose(v1, r1)                           # written in place


def _inplace_cases(call, apply_func):
    g = inplace_graph()
    f = g.ndata["f"]
    call(g, fn.copy_src(src="f", out="m"), fn.sum(msg="m", out="f"), apply_func, False)
    result = g.ndata["f"]
    udf_msg = lambda edges: {"m": edges.src["f"]}  # noqa: E731
    for mf, rf in ((udf_msg, _sum_f), (fn.copy_src(src="f", out="m"), fn.sum(msg="m", out="f")),
                   (udf_msg, fn.sum(msg="m", out="f"))):   # deg bucket, v2v, e2v
        v1 = f.clone()
        g.ndata["f"] = v1
        call(g, mf, rf, apply_func, True)
        r1 = g.ndata["f"]
        assert allclose(r1, result)
        assert allclose(v1, r1)


@pytest.mark.parametrize("apply_func", [_apply2, None])
def test_inplace_snr(apply_func):
    _inplace_cases(lambda g, m, r, a, ip: g.send_and_recv((U, V), m, r, a, inplace=ip), apply_func)


@pytest.mark.parametrize("apply_func", [_apply2, None])
def test_inplace_push(apply_func):
    nodes = th.tensor([0, 3, 4, 9])
    _inplace_cases(lambda g, m, r, a, ip: g.push(nodes, m, r, a, inplace=ip), apply_func)


@pytest.mark.parametrize("apply_func", [_apply2, None])
def test_inplace_pull(apply_func):
    nodes = th.tensor([1, 2, 3, 9])
    _inplace_cases(lambda g, m, r, a, ip: g.pull(nodes, m, r, a, inplace=ip), apply_func)


def test_inplace_apply():
    g = inplace_graph()
    nodes = [1, 2, 3, 9]
    nf = g.ndata["f"]
    g.apply_nodes(lambda n: {"f": n.data["f"] * 2}, nodes)
    new_nf = g.ndata["f"]
    g.ndata["f"] = nf
    g.apply_nodes(lambda n: {"f": n.data["f"] * 2}, nodes, inplace=True)
    assert allclose(nf, new_nf)
    g.ndata["f"] = nf                                     # all nodes: never in place
    g.apply_nodes(lambda n: {"f": n.data["f"] * 2}, inplace=True)
    assert not allclose(nf, g.ndata["f"])
    edges = [3, 5, 7, 10]
    ef = g.edata["e"]
    g.apply_edges(lambda e: {"e": e.data["e"] * 2}, edges)
    new_ef = g.edata["e"]
    g.edata["e"] = ef
    g.apply_edges(lambda e: {"e": e.data["e"] * 2}, edges, inplace=True)
    assert allclose(ef, new_ef)
    g.apply_edges(lambda e: {"e": e.data["e"] * 2}, inplace=True)
    assert not allclose(ef, g.edata["e"])


# ---- group_apply_edges (test_basics.py:628-680) ---------------------------------
@pytest.mark.parametrize("group_by", ["src", "dst"])
def test_group_apply_edges(group_by):
    def edge_udf(edges):
        h = (edges.data["feat"] * (edges.src["h"] + edges.dst["h"])).sum(2)
        return {"norm_feat": th.softmax(h, dim=1)}
    g = DGLGraph()
    g.add_nodes(10)
    g.add_edges(0, [1, 2, 3, 4, 5, 6, 7, 8])
    g.add_edges(1, [2, 3, 4, 6, 7, 8])
    g.add_edges(2, [2, 3, 4, 5, 6, 7, 8])
    g.ndata["h"] = randn(g.number_of_nodes(), D)
    g.edata["feat"] = randn(g.number_of_edges(), D)
    g.group_apply_edges(group_by=group_by, func=edge_udf)
    u, v, eid = g.out_edges(1, form="all") if group_by == "src" else g.in_edges(5, form="all")
    out = g.edges[eid].data["norm_feat"]
    ref = (g.nodes[u].data["h"] + g.nodes[v].data["h"]) * g.edges[eid].data["feat"]
    assert allclose(out, th.softmax(ref.sum(1), dim=0))


def test_group_apply_edges_bucket_ids():
    """test_basics.py:661-680 (GitHub issue 1036): every bucket row holds exactly
    the in-edges of its destination."""
    m = sp.random(10, 10, 0.2, random_state=np.random.RandomState(3))
    g = DGLGraph(m, readonly=True)
    g.ndata["id"] = th.arange(g.number_of_nodes(), device=DEV)
    g.edata["id"] = th.arange(g.number_of_edges(), device=DEV)

    def apply(edges):
        w = edges.data["id"]
        n_nodes, deg = w.shape
        dst = edges.dst["id"][:, 0].cpu()
        eid1 = np.sort(g.in_edges(dst, "eid").numpy().reshape(n_nodes, deg), 1)
        eid2 = np.sort(w.cpu().numpy(), 1)
        assert np.array_equal(eid1, eid2)
        return {"id2": w}
    g.group_apply_edges("dst", apply, inplace=True)
    assert th.equal(g.edata["id2"], g.edata["id"])
