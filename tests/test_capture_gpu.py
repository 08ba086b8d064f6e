"""HIP-graph capture of whole steps through the C ABI: every library call is
stream-ordered (no host sync, scratch from the stream-ordered pool), so a GCN /
fused-GAT forward + backward captured once with torch.cuda.graph replays to the
same bits as the eager step (the kernels are deterministic).  DESIGN.md §6 times
the captured C1 step."""
import pytest
import torch as th

import dgl
from dgl.nn.pytorch import GraphConv, GATConv

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def power_law_graph(n, m, seed):
    g = th.Generator(device=DEV)
    g.manual_seed(seed)
    w = th.arange(1, n + 1, device=DEV, dtype=th.float64).pow(-0.6)
    src = th.multinomial(w.float(), m, replacement=True, generator=g).to(th.int32)
    dst = th.multinomial(w.float(), m, replacement=True, generator=g).to(th.int32)
    ar = th.arange(n, device=DEV, dtype=th.int32)
    return dgl.DGLGraph.from_device_coo(th.cat([src, ar]), th.cat([dst, ar]), n)


def capture(step):
    s = th.cuda.Stream()
    s.wait_stream(th.cuda.current_stream())
    with th.cuda.stream(s):
        for _ in range(2):
            step()
    th.cuda.current_stream().wait_stream(s)
    graph = th.cuda.CUDAGraph()
    with th.cuda.graph(graph):
        step()
    return graph


def test_captured_gcn_step_matches_eager():
    n, m = 2708, 10556
    g = power_law_graph(n, m, 1)
    x = th.randn(n, 1433, device=DEV)
    l1, l2 = GraphConv(1433, 16, activation=th.relu).to(DEV), GraphConv(16, 7).to(DEV)
    params = list(l1.parameters()) + list(l2.parameters())
    y = th.randint(0, 7, (n,), device=DEV)
    out = {}

    def step():
        for p in params:
            p.grad = None if p.grad is None else p.grad.zero_()
        logits = l2(g, l1(g, x))
        th.nn.functional.cross_entropy(logits, y).backward()
        out["logits"] = logits.detach()

    step()
    eager_logits = out["logits"].clone()
    eager_grads = [p.grad.clone() for p in params]
    graph = capture(step)
    for p in params:
        p.grad.fill_(float("nan"))
    graph.replay()
    th.cuda.synchronize()
    assert th.equal(out["logits"], eager_logits)
    for p, e in zip(params, eager_grads):
        assert th.equal(p.grad, e)


def test_captured_fused_gat_matches_eager():
    n, m = 4000, 60000
    g = power_law_graph(n, m, 2)
    x = th.randn(n, 32, device=DEV, requires_grad=True)
    gat = GATConv(32, 8, 4).to(DEV)
    keep = {}

    def step():
        x.grad = None if x.grad is None else x.grad.zero_()
        for p in gat.parameters():
            p.grad = None if p.grad is None else p.grad.zero_()
        h = gat(g, x)
        (h * h).sum().backward()
        keep["h"] = h.detach()

    step()
    eager_h, eager_gx = keep["h"].clone(), x.grad.clone()
    eager_gp = [p.grad.clone() for p in gat.parameters()]
    graph = capture(step)
    x.grad.fill_(float("nan"))
    graph.replay()
    th.cuda.synchronize()
    assert th.equal(keep["h"], eager_h)
    assert th.equal(x.grad, eager_gx)
    for p, e in zip(gat.parameters(), eager_gp):
        assert th.equal(p.grad, e)


def test_captured_relgraphconv_fused_matches_eager():
    """RelGraphConv on the fused layer-1 C entries (tile queues and scratch from the
    stream-ordered pool, the self-loop pass, the 64 x 320 weight-gradient GEMM)
    captured once: replays give the eager step's bits."""
    from dgl.nn.pytorch import RelGraphConv
    n, m, R = 6000, 80000, 4
    g = power_law_graph(n, m, 3)
    gen = th.Generator(device=DEV)
    gen.manual_seed(4)
    et = th.randint(0, R, (g.number_of_edges(),), generator=gen, device=DEV)
    norm = th.rand(g.number_of_edges(), 1, generator=gen, device=DEV)
    x = th.randn(n, 64, device=DEV, requires_grad=True)
    conv = RelGraphConv(64, 64, R, "basis", self_loop=True).to(DEV)
    keep = {}

    def step():
        x.grad = None if x.grad is None else x.grad.zero_()
        for p in conv.parameters():
            p.grad = None if p.grad is None else p.grad.zero_()
        h = conv(g, x, et, norm)
        (h * h).sum().backward()
        keep["h"] = h.detach()

    step()
    assert g._graph.__dict__.get("_rgcn_fused") is not None
    eager_h, eager_gx = keep["h"].clone(), x.grad.clone()
    eager_gp = [p.grad.clone() for p in conv.parameters()]
    graph = capture(step)
    x.grad.fill_(float("nan"))
    graph.replay()
    th.cuda.synchronize()
    assert th.equal(keep["h"], eager_h)
    assert th.equal(x.grad, eager_gx)
    for p, e in zip(conv.parameters(), eager_gp):
        assert th.equal(p.grad, e)
