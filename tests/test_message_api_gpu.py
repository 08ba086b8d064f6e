"""Two-phase send/recv, push, registered default functions and user-defined
message functions on the HIP path.

Known answers restated from the reference's own tests and docstrings:
* tests/compute/test_function.py:5-67 (star graph 0 -> 1..8 -> 9 -> 0 with node
  features 1..10 and edge features [1, 2, 1, 3, ..., 10]): copy_src / copy_edge /
  src_mul_edge summed into every node, through update_all() with registered
  functions and through send() + recv().  The reference reduces with a UDF
  ``sum(mailbox, 1)``; here the builtin ``fn.sum`` (the same arithmetic).
* python/dgl/graph.py:2860-2895 (DGLGraph.recv docstring): messages are consumed
  once received; a received node without a message gets the empty-row value.
"""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn
from dgl._ffi import DGLError

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

STAR_COPY = [10., 1., 1., 1., 1., 1., 1., 1., 1., 44.]
STAR_MUL = [100., 1., 1., 1., 1., 1., 1., 1., 1., 284.]
STAR_EDGE_H = [1., 2., 1., 3., 1., 4., 1., 5., 1., 6., 1., 7., 1., 8., 1., 9., 10.]


def star_graph():
    """test_function.py:5-19."""
    g = dgl.DGLGraph()
    g.add_nodes(10)
    for i in range(1, 9):
        g.add_edge(0, i)
        g.add_edge(i, 9)
    g.add_edge(9, 0)
    g.ndata["h"] = th.arange(1, 11, dtype=th.float32, device=DEV)
    g.edata["h"] = th.tensor(STAR_EDGE_H, device=DEV)
    return g


@pytest.mark.parametrize("msg,expect", [
    (lambda: fn.copy_src(src="h", out="m"), STAR_COPY),
    (lambda: fn.copy_edge(edge="h", out="m"), STAR_COPY),
    (lambda: fn.src_mul_edge(src="h", edge="h", out="m"), STAR_MUL),
])
def test_function_known_answers(msg, expect):
    g = star_graph()
    g.register_message_func(msg())
    g.register_reduce_func(fn.sum(msg="m", out="out"))
    g.update_all()
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(expect))
    g.send()
    g.recv()
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(expect))


def test_function_known_answers_udf_message():
    """Same answers with the message as a UDF (materialised, then copy_e reduced)."""
    g = star_graph()
    g.register_message_func(lambda edges: {"m": edges.src["h"] * edges.data["h"]})
    g.register_reduce_func(fn.sum("m", "out"))
    g.update_all()
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(STAR_MUL))
    g.send(g.edges())
    g.recv(g.nodes())
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(STAR_MUL))


def test_recv_docstring_known_answer():
    """graph.py:2860-2895."""
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.ndata["x"] = th.tensor([[1.], [2.], [3.]], device=DEV)
    g.add_edges([0, 1], [1, 2])
    g.register_message_func(lambda edges: {"m": edges.src["x"]})
    g.register_reduce_func(fn.sum("m", "x"))
    g.send(g.edges())
    g.recv(g.nodes())
    assert th.equal(g.ndata["x"].cpu(), th.tensor([[0.], [1.], [2.]]))
    g.recv(g.nodes())  # messages were consumed: nothing happens
    assert th.equal(g.ndata["x"].cpu(), th.tensor([[0.], [1.], [2.]]))


def test_send_partial_then_recv_subset():
    """Messages sent on some edges are received only by the requested nodes;
    the others stay pending until their own recv."""
    g = star_graph()
    g.register_message_func(fn.copy_src("h", "m"))
    g.register_reduce_func(fn.sum("m", "out"))
    # edges 0->1 (eid 0), 0->2 (eid 2), 1->9 (eid 1), 2->9 (eid 3), 9->0 (eid 16)
    g.send([0, 1, 2, 3, 16])
    g.recv([9])
    out = g.ndata["out"].cpu()
    assert out[9] == 2. + 3.  # h[1] + h[2]
    assert th.all(out[:9] == 0)
    g.recv([0, 1, 2, 5])
    out = g.ndata["out"].cpu()
    assert out[0] == 10. and out[1] == 1. and out[2] == 1. and out[5] == 0.
    assert out[9] == 5.
    g.recv()  # everything consumed
    assert th.equal(g.ndata["out"].cpu(), out)


def test_send_recv_max_and_apply():
    g = star_graph()
    g.send(message_func=fn.copy_src("h", "m"))
    g.recv(reduce_func=fn.max("m", "mx"),
           apply_node_func=lambda nodes: {"mx": nodes.data["mx"] * 2})
    assert th.equal(g.ndata["mx"].cpu(), 2 * th.tensor([10., 1., 1., 1., 1., 1., 1., 1., 1., 9.]))


def test_push_and_pull_known_answers():
    g = star_graph()
    g.push([0], fn.copy_src("h", "m"), fn.sum("m", "out"))
    out = g.ndata["out"].cpu()
    assert th.equal(out, th.tensor([0., 1., 1., 1., 1., 1., 1., 1., 1., 0.]))
    g.pull([9, 0], fn.copy_src("h", "m"), fn.sum("m", "out"))
    out = g.ndata["out"].cpu()
    assert out[9] == 44. and out[0] == 10. and out[1] == 1.
    # pull on a node without in-edges downgrades to apply_nodes (scheduler.py:472-476)
    g2 = dgl.DGLGraph()
    g2.add_nodes(2)
    g2.add_edge(0, 1)
    g2.ndata["h"] = th.tensor([1., 2.], device=DEV)
    g2.pull([0], fn.copy_src("h", "m"), fn.sum("m", "h"),
            lambda nodes: {"h": nodes.data["h"] + 5})
    assert th.equal(g2.ndata["h"].cpu(), th.tensor([6., 2.]))


def test_udf_message_matches_builtin_with_grad():
    """u_mul_e as a UDF message == the builtin kernel, values and gradients."""
    rng = np.random.default_rng(5)
    n, m, f = 300, 4000, 16
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    x = th.randn(n, f, device=DEV)
    w = th.randn(m, f, device=DEV)
    res = []
    for udf in (False, True):
        g = dgl.DGLGraph()
        g.add_nodes(n)
        g.add_edges(src, dst)
        xs, ws = x.clone().requires_grad_(), w.clone().requires_grad_()
        g.ndata["x"], g.edata["w"] = xs, ws
        mf = (lambda e: {"m": e.src["x"] * e.data["w"]}) if udf else fn.u_mul_e("x", "w", "m")
        g.update_all(mf, [fn.sum("m", "s"), fn.mean("m", "a")])
        (g.ndata["s"].sum() + (g.ndata["a"] ** 2).sum()).backward()
        res.append((g.ndata["s"].detach(), g.ndata["a"].detach(), xs.grad, ws.grad))
    for a, b in zip(*res):
        assert th.allclose(a, b, rtol=1e-4, atol=1e-4)


def reducer_both(nodes):
    """test_function.py:21-22, the reference's own reduce UDF."""
    return {"out": th.sum(nodes.mailbox["m"], 1)}


@pytest.mark.parametrize("msg,expect", [
    (lambda: fn.copy_src(src="h", out="m"), STAR_COPY),
    (lambda: fn.copy_edge(edge="h", out="m"), STAR_COPY),
    (lambda: fn.src_mul_edge(src="h", edge="h", out="m"), STAR_MUL),
])
def test_function_known_answers_reduce_udf(msg, expect):
    """test_function.py:24-67 verbatim in structure: builtin message + the reference's
    UDF reducer (degree bucketing), update_all() and send() + recv()."""
    g = star_graph()
    g.register_message_func(msg())
    g.register_reduce_func(reducer_both)
    g.update_all()
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(expect))
    g.send()
    g.recv()
    assert th.equal(g.ndata.pop("out").cpu(), th.tensor(expect))


def test_recv_docstring_known_answer_reduce_udf():
    """graph.py:2860-2895 with the docstring's own UDFs."""
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.ndata["x"] = th.tensor([[1.], [2.], [3.]], device=DEV)
    g.add_edges([0, 1], [1, 2])
    g.register_message_func(lambda edges: {"m": edges.src["x"]})
    g.register_reduce_func(lambda nodes: {"x": nodes.mailbox["m"].sum(1)})
    g.send(g.edges())
    g.recv(g.nodes())
    assert th.equal(g.ndata["x"].cpu(), th.tensor([[0.], [1.], [2.]]))
    g.recv(g.nodes())
    assert th.equal(g.ndata["x"].cpu(), th.tensor([[0.], [1.], [2.]]))


@pytest.mark.parametrize("red", ["sum", "max", "min", "mean", "prod"])
def test_degree_bucketing_matches_builtin(red):
    """A reduce UDF over mailboxes == the builtin reducer (nodes with in-edges; the
    UDF path leaves zero-in-degree rows at 0), values and gradients."""
    rng = np.random.default_rng(11)
    n, m, f = 200, 1500, 8
    src, dst = rng.integers(0, n, m), (rng.pareto(1.0, m) * 10).astype(np.int64) % n
    if red in ("max", "min"):
        # no repeated (u, v) pairs: a tie sends the builtin's gradient to every tied
        # edge (cpu/functor.h:36-38) but torch.max's to one of them
        pairs = np.unique(np.stack([src, dst], 1), axis=0)
        src, dst = pairs[rng.permutation(len(pairs))].T
    x = th.rand(n, f, device=DEV) + 0.5
    udf = {"sum": lambda nb: {"o": nb.mailbox["m"].sum(1)},
           "max": lambda nb: {"o": nb.mailbox["m"].max(1)[0]},
           "min": lambda nb: {"o": nb.mailbox["m"].min(1)[0]},
           "mean": lambda nb: {"o": nb.mailbox["m"].mean(1)},
           "prod": lambda nb: {"o": nb.mailbox["m"].prod(1)}}[red]
    outs = []
    for reduce_func in (getattr(fn, red)("m", "o"), udf):
        g = dgl.DGLGraph()
        g.add_nodes(n)
        g.add_edges(src, dst)
        xs = x.clone().requires_grad_()
        g.ndata["x"] = xs
        g.update_all(fn.copy_u("x", "m"), reduce_func)
        o = g.ndata["o"]
        o.backward(th.ones_like(o))
        outs.append((o.detach(), xs.grad))
    has = th.as_tensor(np.bincount(dst, minlength=n) > 0, device=DEV)
    tol = 1e-2 if red == "prod" else 1e-4
    assert th.allclose(outs[0][0][has], outs[1][0][has], rtol=tol, atol=tol)
    assert th.all(outs[1][0][~has] == 0)
    assert th.allclose(outs[0][1], outs[1][1], rtol=tol, atol=tol)


def test_reduce_udf_pull_and_mailbox_order():
    """Mailboxes list a node's messages in edge-id order (scheduler.cc:20-24)."""
    g = dgl.DGLGraph()
    g.add_nodes(4)
    g.add_edges([3, 1, 2, 0, 3], [0, 0, 0, 1, 2])
    g.ndata["x"] = th.tensor([10., 20., 30., 40.], device=DEV).view(4, 1)
    seen = {}

    def red(nodes):
        seen[nodes.mailbox["m"].shape[1]] = nodes.mailbox["m"][..., 0].cpu()
        return {"y": nodes.mailbox["m"][:, 0] * 1000 + nodes.mailbox["m"][:, -1]}
    g.pull([0, 2, 3], fn.copy_u("x", "m"), red)
    assert th.equal(seen[3], th.tensor([[40., 20., 30.]]))
    y = g.ndata["y"].cpu().view(-1)
    assert y[0] == 40 * 1000 + 30 and y[2] == 40 * 1000 + 40 and y[3] == 0 and y[1] == 0


def test_missing_functions_raise():
    g = star_graph()
    with pytest.raises(DGLError):
        g.update_all()
    with pytest.raises(DGLError):
        g.send()
    g.register_message_func(fn.copy_src("h", "m"))
    with pytest.raises(DGLError):
        g.update_all()


def test_saved_graph_runs_update_all(tmp_path):
    """save_graphs of device features (written as CPU arrays, ndarray.h:415-427), then
    load_graphs -> update_all on the GPU: the known answers of the star graph again."""
    from dgl.data.utils import save_graphs, load_graphs
    g = star_graph()
    path = str(tmp_path / "star.bin")
    save_graphs(path, [g], {"y": th.ones(1, device=DEV)})
    (h,), labels = load_graphs(path)
    assert h.ndata["h"].device.type == "cpu" and labels["y"].device.type == "cpu"
    h = h.to(DEV)
    h.update_all(fn.src_mul_edge(src="h", edge="h", out="m"), fn.sum(msg="m", out="out"))
    assert th.equal(h.ndata["out"].cpu(), th.tensor(STAR_MUL))
