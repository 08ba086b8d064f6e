"""R-GCN on the typed-gather path vs fp64 restatements of the hack's layer
kernels (binary_reduce_impl.cu:913-1246) and of RelGraphConv's per-edge bmm
message function (nn/pytorch/conv/relgraphconv.py:125-150)."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
from dgl.nn.pytorch import RelGraphConv
from graphs import powerlaw

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def typed_graph(n=3000, m=40000, R=4, seed=0):
    src, dst, n = powerlaw(n, m, seed=seed)
    et = np.random.default_rng(seed).integers(0, R, len(src))
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges_with_type(src, dst, et)
    return g, src, dst, et, n


def dense_typed(src, dst, et, n, y, norm):
    """out[v] = sum_e norm_e * y[t_e, u_e]   (y: (R, N, F))"""
    s, d, t = (th.from_numpy(a).to(DEV) for a in (src, dst, et))
    msg = y[t, s] * (norm if norm is not None else 1.0)
    return th.zeros(n, y.shape[2], dtype=y.dtype, device=DEV).index_add(0, d, msg)


@pytest.mark.parametrize("F", [16, 7])
def test_rgcn_layer0(F):
    g, src, dst, et, n = typed_graph()
    R = 4
    W = th.randn(R, n, F, device=DEV, requires_grad=True)
    norm = th.rand(len(src), 1, device=DEV, requires_grad=True)
    out = B.rgcn_layer0(g, W, norm)
    go = th.randn_like(out)
    gW, gn = th.autograd.grad(out, (W, norm), go)
    Wd, nd = W.detach().double().requires_grad_(), norm.detach().double().requires_grad_()
    ref = dense_typed(src, dst, et, n, Wd, nd)
    rW, rn = th.autograd.grad(ref, (Wd, nd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    assert th.allclose(gW.double(), rW, rtol=1e-4, atol=1e-4)
    assert th.allclose(gn.double(), rn, rtol=1e-4, atol=1e-4)


def test_rgcn_layer1():
    g, src, dst, et, n = typed_graph(seed=1)
    R, fin, fout = 4, 24, 16
    x = th.randn(n, fin, device=DEV, requires_grad=True)
    W = th.randn(R, fin, fout, device=DEV, requires_grad=True)
    norm = th.rand(len(src), 1, device=DEV)
    out = B.rgcn_layer1(g, x, W, norm)
    go = th.randn_like(out)
    gx, gW = th.autograd.grad(out, (x, W), go)
    xd, Wd = x.detach().double().requires_grad_(), W.detach().double().requires_grad_()
    ref = dense_typed(src, dst, et, n, th.matmul(xd.unsqueeze(0), Wd), norm.double())
    rx, rW = th.autograd.grad(ref, (xd, Wd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-3)
    assert th.allclose(gx.double(), rx, rtol=1e-3, atol=1e-3)
    assert th.allclose(gW.double(), rW, rtol=1e-3, atol=1e-2)


def ref_relgraphconv(conv, src, dst, x, et, norm, n):
    """relgraphconv.py:125-150 + update_all(sum), in fp64."""
    s, d, t = (th.from_numpy(a).to(DEV) for a in (src, dst, et))
    if conv.regularizer == "basis":
        W = conv._relation_weights().double()
        if x.dtype == th.int64:
            msg = W[t, x[s]]
        else:
            msg = th.bmm(x.double()[s].unsqueeze(1), W[t]).squeeze(1)
    else:
        w = conv.weight.double().index_select(0, t).view(-1, conv.submat_in, conv.submat_out)
        node = x.double()[s].view(-1, 1, conv.submat_in)
        msg = th.bmm(node, w).view(-1, conv.out_feat)
    if norm is not None:
        msg = msg * norm.double()
    out = th.zeros(n, conv.out_feat, dtype=th.float64, device=DEV).index_add(0, d, msg)
    if conv.bias:
        out = out + conv.h_bias.double()
    if conv.self_loop:
        out = out + (conv.loop_weight.double()[x] if x.dtype == th.int64 else x.double() @ conv.loop_weight.double())
    return out


@pytest.mark.parametrize("reg,bases,ids,loop", [("basis", 2, False, False), ("basis", None, True, True),
                                                ("bdd", 4, False, True)])
def test_relgraphconv(reg, bases, ids, loop):
    g, src, dst, et, n = typed_graph(seed=2)
    R = 4
    th.manual_seed(0)
    conv = RelGraphConv(n if ids else 32, 16, R, regularizer=reg, num_bases=bases,
                        self_loop=loop).to(DEV)
    x = th.arange(n, device=DEV) if ids else th.randn(n, 32, device=DEV)
    etypes = th.from_numpy(et).to(DEV)
    norm = th.rand(len(src), 1, device=DEV)
    out = conv(g, x, etypes, norm)
    ref = ref_relgraphconv(conv, src, dst, x, et, norm, n)
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-3)
    out.pow(2).sum().backward()
    grads = [p.grad.clone() for p in conv.parameters()]
    conv.zero_grad()
    ref.pow(2).sum().backward()
    for a, p in zip(grads, conv.parameters()):
        assert th.allclose(a, p.grad, rtol=1e-3, atol=1e-2)


def test_constant_norm_position_cache_follows_the_tensor():
    """A constant norm is streamed from a cached copy in in-CSR position order
    (ImmutableGraphIndex.position_operand); an in-place update or another tensor
    must not reuse a stale copy, and a norm that needs a gradient takes the
    edge-id path."""
    g, src, dst, et, n = typed_graph(seed=4)
    R, fin, fout = 4, 8, 8
    x = th.randn(n, fin, device=DEV)
    W = th.randn(R, fin, fout, device=DEV)
    norm = th.rand(len(src), 1, device=DEV)
    a = B.rgcn_layer1(g, x, W, norm)
    norm.mul_(2.0)
    b = B.rgcn_layer1(g, x, W, norm)
    assert th.allclose(b, 2 * a, rtol=1e-5, atol=1e-5)
    c = B.rgcn_layer1(g, x, W, norm / 2)
    assert th.allclose(c, a, rtol=1e-5, atol=1e-5)
    # a temporary norm per call (freed in between, so the allocator may hand the
    # next one the same address) must never hit a stale cached copy
    outs = [B.rgcn_layer1(g, x, W, th.full((len(src), 1), float(k), device=DEV))
            for k in (1, 2, 3)]
    assert th.allclose(outs[1], 2 * outs[0], rtol=1e-5, atol=1e-5)
    assert th.allclose(outs[2], 3 * outs[0], rtol=1e-4, atol=1e-4)  # x3 rounds
    ng = norm.clone().requires_grad_()
    d = B.rgcn_layer1(g, x, W, ng)
    assert th.equal(d, b)
    (gn,) = th.autograd.grad(d.sum(), (ng,))
    assert gn.shape == ng.shape


@pytest.mark.parametrize("R,bases,loop,act", [(4, None, True, False), (4, 2, False, True),
                                              (2, None, True, True), (3, 2, False, False)])
def test_relgraphconv_fused_route(R, bases, loop, act):
    """64 -> 64 layers with a constant norm run on the fused layer-1 C entries
    (dgl.backend.rgcn_fused_route, bias and self-loop in the output pass): equal to
    the fp64 per-edge bmm restatement and to the GEMM + typed-gather path, forward
    and every parameter / input gradient."""
    g, src, dst, et, n = typed_graph(seed=5, R=R)
    th.manual_seed(1)
    conv = RelGraphConv(64, 64, R, "basis", num_bases=bases, self_loop=loop,
                        activation=th.tanh if act else None).to(DEV)
    x = th.randn(n, 64, device=DEV, requires_grad=True)
    etypes = th.from_numpy(et).to(DEV)
    norm = th.rand(len(src), 1, device=DEV)
    out = conv(g, x, etypes, norm)
    assert g._graph.__dict__.get("_rgcn_fused") is not None  # the fused route ran
    ref = ref_relgraphconv(conv, src, dst, x.detach(), et, norm, n)
    if act:
        ref = th.tanh(ref)
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    go = th.randn_like(out)
    params = [x] + list(conv.parameters())
    grads = th.autograd.grad(out, params, go)
    conv.use_fused = False
    out2 = conv(g, x, etypes, norm)
    grads2 = th.autograd.grad(out2, params, go)
    assert th.allclose(out, out2, rtol=1e-4, atol=1e-4)  # fp32, other summation order
    for a, b in zip(grads, grads2):  # long fp32 sums in other orders: scaled bound
        assert (a - b).abs().max().item() <= 1e-3 + 1e-4 * b.abs().max().item()
    # the fp64 gradients
    xd = x.detach().double().requires_grad_()
    conv64 = RelGraphConv(64, 64, R, "basis", num_bases=bases, self_loop=loop,
                          activation=th.tanh if act else None).to(DEV).double()
    conv64.load_state_dict({k: v.double() for k, v in conv.state_dict().items()})
    ref = ref_relgraphconv(conv64, src, dst, xd, et, norm, n)
    if act:
        ref = th.tanh(ref)
    rgrads = th.autograd.grad(ref, [xd] + list(conv64.parameters()), go.double())
    for a, b in zip(grads, rgrads):
        mass = b.abs().max().item()
        assert (a.double() - b).abs().max().item() <= 1e-3 + 1e-4 * mass


def test_relgraphconv_fused_state_follows_the_tensors():
    """The fused route's prepared state is keyed on etypes and its version counter:
    an in-place update of norm or a new norm per call re-gathers the cached norm
    copies (same state), new etypes rebuild it (the old state released first, one
    alive); a norm that needs a gradient and 32-wide layers keep the typed-gather path."""
    import gc
    from dgl import kernel as K
    g, src, dst, et, n = typed_graph(seed=6)
    R = 4
    th.manual_seed(2)
    conv = RelGraphConv(64, 64, R, "basis", bias=False).to(DEV)
    x = th.randn(n, 64, device=DEV)
    etypes = th.from_numpy(et).to(DEV)
    norm = th.rand(len(src), 1, device=DEV)
    gc.collect()
    live = K.RgcnState.live
    with th.no_grad():
        a = conv(g, x, etypes, norm)
        st = g._graph.__dict__["_rgcn_fused"][1].__dict__["_rgcn_state"]
        assert K.RgcnState.live == live + 1
        norm.mul_(2.0)
        b = conv(g, x, etypes, norm)
        assert th.allclose(b, 2 * a, rtol=1e-5, atol=1e-5)
        outs = [conv(g, x, etypes, th.full((len(src), 1), float(k), device=DEV)) for k in (1, 2, 3)]
        assert th.allclose(outs[1], 2 * outs[0], rtol=1e-5, atol=1e-5)
        assert th.allclose(outs[2], 3 * outs[0], rtol=1e-4, atol=1e-4)
        assert g._graph.__dict__["_rgcn_fused"][1].__dict__["_rgcn_state"] is st
        et2 = (etypes + 1) % R
        c = conv(g, x, et2, norm)
        assert K.RgcnState.live == live + 1 and not st._fin.alive
        conv.use_fused = False
        c2 = conv(g, x, et2, norm)
        assert th.allclose(c, c2, rtol=1e-4, atol=1e-4)
        conv.use_fused = True
    ng = norm.clone().requires_grad_()
    g._graph.__dict__["_rgcn_fused"] = None
    d = conv(g, x, etypes, ng)
    assert g._graph.__dict__.get("_rgcn_fused") is None
    (gn,) = th.autograd.grad(d.sum(), (ng,))
    assert gn.shape == ng.shape
    narrow = RelGraphConv(32, 64, R, "basis").to(DEV)
    narrow(g, th.randn(n, 32, device=DEV), etypes, norm)
    assert g._graph.__dict__.get("_rgcn_fused") is None


def test_relgraphconv_fused_first_layer_param_grads():
    """A first layer (input without gradient): the fused backward skips the input
    gradient; the parameter gradients equal the GEMM + typed-gather path's."""
    g, src, dst, et, n = typed_graph(seed=8)
    th.manual_seed(3)
    conv = RelGraphConv(64, 64, 4, "basis", num_bases=2, self_loop=True).to(DEV)
    x = th.randn(n, 64, device=DEV)
    etypes = th.from_numpy(et).to(DEV)
    norm = th.rand(len(src), 1, device=DEV)
    go = th.randn(n, 64, device=DEV)
    grads = th.autograd.grad(conv(g, x, etypes, norm), list(conv.parameters()), go)
    assert g._graph.__dict__.get("_rgcn_fused") is not None
    conv.use_fused = False
    grads2 = th.autograd.grad(conv(g, x, etypes, norm), list(conv.parameters()), go)
    for a, b in zip(grads, grads2):
        assert (a - b).abs().max().item() <= 1e-3 + 1e-4 * b.abs().max().item()


def test_relgraphconv_fused_noncontiguous_norm_refreshes_once(monkeypatch):
    """A non-contiguous norm (a column of a wider tensor) is flattened once per (tensor,
    version) and the copy reused (dgl.backend._flat_norm), so the prepared state's norm
    copies are re-gathered (DGLMIRgcnRefreshNorm) once, not on every call; an in-place
    update still refreshes them."""
    from dgl import _ffi
    g, src, dst, et, n = typed_graph(seed=9)
    R = 4
    th.manual_seed(4)
    conv = RelGraphConv(64, 64, R, "basis").to(DEV)
    x = th.randn(n, 64, device=DEV)
    etypes = th.from_numpy(et).to(DEV)
    wide = th.rand(len(src), 3, device=DEV)
    norm = wide[:, 1:2]  # (E, 1), stride 3: not contiguous
    assert not norm.is_contiguous()
    lib = _ffi.lib()
    orig = lib.DGLMIRgcnRefreshNorm
    calls = []
    monkeypatch.setattr(lib, "DGLMIRgcnRefreshNorm", lambda *a: calls.append(1) or orig(*a))
    with th.no_grad():
        a = conv(g, x, etypes, norm)
        first = len(calls)
        for _ in range(3):
            b = conv(g, x, etypes, norm)
        assert len(calls) == first  # no re-gather for the same tensor and version
        assert th.equal(a, b)
        wide.mul_(2.0)  # the same view, a new version
        c = conv(g, x, etypes, norm)
        assert len(calls) == first + 1
    ref = conv(g, x, etypes, norm.contiguous())
    assert th.allclose(c, ref, rtol=1e-5, atol=1e-5)
