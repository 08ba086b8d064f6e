"""Heterograph message passing on the MI355X (heterograph.py:3570-3656,
nn/pytorch/hetero.py:112-170): the reference's own multi_update_all example as a
known answer, every cross-type reducer, the fused cross-type sum against the
per-relation path, HeteroGraphConv against per-relation modules, GATConv on a
bipartite relation."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn
import dgl.nn.pytorch as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_multi_update_all_docstring_known_answer():
    """heterograph.py:3611-3625 (docstring example) -> user h = [[0], [4]]."""
    g1 = dgl.graph([(0, 1), (1, 1)], "user", "follows")
    g2 = dgl.bipartite([(0, 1)], "game", "attracts", "user")
    g = dgl.hetero_from_relations([g1, g2])
    g.nodes["user"].data["h"] = th.tensor([[1.], [2.]], device=DEV)
    g.nodes["game"].data["h"] = th.tensor([[1.]], device=DEV)
    g.multi_update_all({"follows": (fn.copy_src("h", "m"), fn.sum("m", "h")),
                        "attracts": (fn.copy_src("h", "m"), fn.sum("m", "h"))}, "sum")
    assert g.nodes["user"].data["h"].cpu().tolist() == [[0.0], [4.0]]


def _rand_hetero(seed=0, f=16):
    rs = np.random.RandomState(seed)
    nu, ng = 3000, 800

    def rel(ns, nd, m):
        return rs.randint(0, ns, m), rs.randint(0, nd, m)
    g = dgl.heterograph({("user", "follows", "user"): rel(nu, nu, 40000),
                         ("game", "attracts", "user"): rel(ng, nu, 15000),
                         ("user", "plays", "game"): rel(nu, ng, 20000),
                         ("user", "likes", "user"): rel(nu, nu, 10000)},
                        {"user": nu, "game": ng})
    g.nodes["user"].data["h"] = th.from_numpy(rs.randn(nu, f).astype(np.float32)).to(DEV)
    g.nodes["game"].data["h"] = th.from_numpy(rs.randn(ng, f).astype(np.float32)).to(DEV)
    return g


def _per_relation(g, etypes):
    outs = {}
    for e in etypes:
        c = g.to_canonical_etype(e)
        rel = g[c].local_var()
        rel.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
        outs.setdefault(c[2], []).append(rel.dstdata["o"])
    return outs


@pytest.mark.parametrize("cross", ["sum", "max", "min", "mean", "stack"])
def test_multi_update_all_cross_reducers(cross):
    g = _rand_hetero()
    etypes = ["follows", "attracts", "plays", "likes"]
    ref = _per_relation(g, etypes)
    g.multi_update_all({e: (fn.copy_src("h", "m"), fn.sum("m", "o")) for e in etypes}, cross)
    for nt, outs in ref.items():
        if cross == "stack":
            want = th.stack(outs, 1)
        elif cross == "sum":
            want = sum(o.double() for o in outs).float()
        else:
            want = getattr(th.stack(outs, 0), cross)(0)
            want = want[0] if isinstance(want, tuple) else want
        got = g.nodes[nt].data["o"]
        assert got.shape == want.shape
        assert th.allclose(got, want, rtol=1e-5, atol=1e-5), (cross, nt)


def test_fused_cross_sum_is_one_kernel_over_merged_relations():
    """The fused sum (merged block, one SpMM) equals per-relation SpMMs + sum,
    including the gradient w.r.t. every source table."""
    g = _rand_hetero(seed=3)
    etypes = ["follows", "attracts", "likes"]
    xu = g.nodes["user"].data["h"].clone().requires_grad_()
    xg = g.nodes["game"].data["h"].clone().requires_grad_()
    g.nodes["user"].data["h"] = xu
    g.nodes["game"].data["h"] = xg
    g.multi_update_all({e: (fn.copy_src("h", "m"), fn.sum("m", "o")) for e in etypes}, "sum")
    assert len(g._fused) == 1
    out = g.nodes["user"].data["o"]
    go = th.randn_like(out)
    out.backward(go)
    # fp64 reference from the edge lists
    want = th.zeros(out.shape, dtype=th.float64)
    gu = th.zeros(xu.shape, dtype=th.float64)
    gg = th.zeros(xg.shape, dtype=th.float64)
    for e in etypes:
        s, _, d = g.to_canonical_etype(e)
        u, v = g.edges(etype=e)
        x = (xu if s == "user" else xg).detach().double().cpu()
        want.index_add_(0, v, x[u])
        (gu if s == "user" else gg).index_add_(0, u, go.double().cpu()[v])
    assert th.allclose(out.double().cpu(), want, rtol=1e-5, atol=1e-4)
    assert th.allclose(xu.grad.double().cpu(), gu, rtol=1e-5, atol=1e-4)
    assert th.allclose(xg.grad.double().cpu(), gg, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("agg", ["sum", "mean", "stack"])
def test_hetero_graph_conv(agg):
    g = _rand_hetero(seed=5)
    th.manual_seed(0)
    mods = {e: nn.GraphConv(16, 8) for e in ["follows", "attracts", "plays", "likes"]}
    conv = nn.HeteroGraphConv(mods, aggregate=agg).to(DEV)
    inputs = {"user": g.nodes["user"].data["h"], "game": g.nodes["game"].data["h"]}
    out = conv(g, inputs)
    assert set(out) == {"user", "game"}
    per = {}
    for c in g.canonical_etypes:
        per.setdefault(c[2], []).append(conv.mods[c[1]](g[c], inputs[c[0]]))
    for nt, outs in per.items():
        want = {"sum": lambda t: sum(t), "mean": lambda t: th.stack(t, 0).mean(0),
                "stack": lambda t: th.stack(t, 1)}[agg](outs)
        assert th.allclose(out[nt], want, rtol=1e-5, atol=1e-5)
    # GraphConv on a bipartite relation vs dense A X W with both norms
    rel = g["user", "plays", "game"]
    u, v = g.edges(etype="plays")
    A = th.zeros(800, 3000, dtype=th.float64).index_put_((v, u), th.ones(len(u), dtype=th.float64),
                                                         accumulate=True)
    dout = A.sum(0).clamp(min=1)
    din = A.sum(1).clamp(min=1)
    x = inputs["user"].double().cpu()
    m = conv.mods["plays"]
    y = (A @ ((x * dout.pow(-0.5)[:, None]) @ m.weight.double().cpu())) * din.pow(-0.5)[:, None]
    y = y + m.bias.double().cpu()
    assert th.allclose(m(rel, inputs["user"]).double().cpu(), y, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("use_fused", [True, False])
def test_gat_conv_on_bipartite_relation(use_fused):
    g = _rand_hetero(seed=7)
    th.manual_seed(1)
    gat = nn.GATConv((16, 16), 8, 4).to(DEV)
    gat.use_fused = use_fused
    rel = g["user", "plays", "game"]
    out = gat(rel, (g.nodes["user"].data["h"], g.nodes["game"].data["h"]))
    assert out.shape == (800, 4, 8)
    gat.use_fused = not use_fused
    out2 = gat(rel, (g.nodes["user"].data["h"], g.nodes["game"].data["h"]))
    assert th.allclose(out, out2, rtol=1e-4, atol=1e-5)


def _test_heterograph():
    """tests/compute/test_heterograph.py:12-32 (the wishes relation from its edge
    list: networkx is not installed here)."""
    import scipy.sparse as ssp
    plays = ssp.coo_matrix(([1, 1, 1, 1], ([0, 1, 2, 1], [0, 0, 1, 1])))
    follows_g = dgl.graph([(0, 1), (1, 2)], "user", "follows")
    plays_g = dgl.bipartite(plays, "user", "plays", "game")
    wishes_g = dgl.bipartite([(0, 1), (2, 0)], "user", "wishes", "game")
    develops_g = dgl.bipartite([(0, 0), (1, 1)], "developer", "develops", "game")
    return dgl.hetero_from_relations([follows_g, plays_g, wishes_g, develops_g])


def test_relation_updates_known_answers():
    """test_heterograph.py:1313-1359: update_all / send_and_recv / send + recv / pull
    / push on the (user, plays, game) relation, builtin and UDF message / reduce,
    with and without an apply function."""
    import itertools

    def msg_func(edges):
        return {"m": edges.src["h"]}

    def reduce_func(nodes):
        return {"y": nodes.mailbox["m"].sum(1)}

    def apply_func(nodes):
        return {"y": nodes.data["y"] * 2}
    g = _test_heterograph()
    x = th.randn(3, 5, device=DEV)
    g.nodes["user"].data["h"] = x
    close = lambda a, b: th.allclose(a, b, rtol=1e-6, atol=1e-6)  # noqa: E731
    for msg, red, apply in itertools.product([fn.copy_u("h", "m"), msg_func],
                                             [fn.sum("m", "y"), reduce_func],
                                             [None, apply_func]):
        k = 1 if apply is None else 2
        g["user", "plays", "game"].update_all(msg, red, apply)
        y = g.nodes["game"].data["y"]
        assert close(y[0], (x[0] + x[1]) * k) and close(y[1], (x[1] + x[2]) * k)
        del g.nodes["game"].data["y"]
        g["user", "plays", "game"].send_and_recv(([0, 1, 2], [0, 1, 1]), msg, red, apply)
        y = g.nodes["game"].data["y"]
        assert close(y[0], x[0] * k) and close(y[1], (x[1] + x[2]) * k)
        del g.nodes["game"].data["y"]
        plays_g = g["user", "plays", "game"]
        plays_g.send(([0, 1, 2], [0, 1, 1]), msg)
        plays_g.recv([0, 1], red, apply)
        y = g.nodes["game"].data["y"]
        assert close(y[0], x[0] * k) and close(y[1], (x[1] + x[2]) * k)
        del g.nodes["game"].data["y"]
        g["user", "plays", "game"].pull(0, msg, red, apply)
        y = g.nodes["game"].data["y"]
        assert close(y[0], (x[0] + x[1]) * k)
        del g.nodes["game"].data["y"]
        g["user", "plays", "game"].push(0, msg, red, apply)
        y = g.nodes["game"].data["y"]
        assert close(y[0], x[0] * k)
        del g.nodes["game"].data["y"]


def test_multi_update_all_backward_known_answer():
    """test_heterograph.py:1361-1376: plays + wishes summed into games, ones as the
    upstream gradient -> every user row gets 2."""
    g = _test_heterograph()
    x = th.randn(3, 5, device=DEV, requires_grad=True)
    g.nodes["user"].data["h"] = x
    g.multi_update_all({"plays": (fn.copy_u("h", "m"), fn.sum("m", "y")),
                        "wishes": (fn.copy_u("h", "m"), fn.sum("m", "y"))}, "sum")
    y = g.nodes["game"].data["y"]
    y.backward(th.ones_like(y))
    assert th.equal(x.grad.cpu(), th.full((3, 5), 2.))


def test_stack_reduce_shapes():
    """test_heterograph.py:1463-1487."""
    g = _test_heterograph()
    g.nodes["user"].data["h"] = th.randn(3, 200, device=DEV)

    def mfunc(edges):
        return {"m": edges.src["h"]}
    g.multi_update_all({"plays": (mfunc, lambda n: {"y": n.mailbox["m"].sum(1)}),
                        "wishes": (mfunc, lambda n: {"y": n.mailbox["m"].max(1)[0]})}, "stack")
    assert tuple(g.nodes["game"].data["y"].shape) == (g.number_of_nodes("game"), 2, 200)
    g.multi_update_all({"plays": (mfunc, lambda n: {"y": n.mailbox["m"].sum(1)})}, "stack")
    assert tuple(g.nodes["game"].data["y"].shape) == (g.number_of_nodes("game"), 1, 200)
