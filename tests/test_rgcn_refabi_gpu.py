"""The hack's R-GCN PackedFuncs in the reference's own argument lists
(``_CAPI_DGLRgcnLayer0(G, weight, norm, ret)``, ``…Layer0Backward(G, grad_out, norm,
grad_weight)``, ``…Layer1(G, hidden, weight, norm, ret)``, ``…Layer1Backward(G,
hidden, weight, norm, grad_out, grad_hidden, grad_weight)``; reference
``src/kernel/binary_reduce.cc:412-450``, ``python/dgl/kernel.py:159-170``).  The graph
carries its edge types, as the reference's graph object does
(``Graph::AddEdgesWithType`` / ``GetCsrSortedByEdgeType``, ``src/graph/graph.cc:690-746``;
here ``DGLGraph.add_edges_with_type`` fills ``DGLMIGraph.etypes``).

``RgcnFirstLayer`` / ``RgcnSecondLayer`` below restate the reference's caller
(``python/dgl/backend/pytorch/tensor.py:440-495``) with the kernel calls bound to
libdglmi in the same order, and their results are checked against the restatement of
the hack's CUDA kernels (``oracle/hack_ref.c``).  Tolerance as in
``test_hack_oracle_gpu.py``: |product - oracle| <= 1e-5 + 2e-5 * (sum of absolute
terms).  The layer-0 backward is compared with the exact sum (the hack's store drops
repeated (source, relation) pairs, ``binary_reduce_impl.cu:1004``), and the layer-1
weight gradient the reference's caller drops (``tensor.py:493``) is checked too."""
import ctypes

import numpy as np
import pytest
import torch as th

import dgl
from dgl import _ffi
from dgl import kernel as K
from graphs import powerlaw
from oracle import oracle as O
from test_hack_oracle_gpu import _close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class RgcnFirstLayer(th.autograd.Function):
    """tensor.py:440-461."""

    @staticmethod
    def forward(ctx, graph, weight, norm, ret):
        ctx.backward_cache = graph, weight.size(), norm
        K.rgcn_layer0(graph, weight, norm, ret)
        return ret

    @staticmethod
    def backward(ctx, gradout):
        graph, weight_size, norm = ctx.backward_cache
        grad_weight = th.zeros(weight_size, dtype=norm.dtype, device=norm.device)
        K.rgcn_layer0_backward(graph, gradout.contiguous(), norm, grad_weight)
        return None, grad_weight, None, None


def rgcn_layer0(graph, weight, norm):
    """tensor.py:463-466 (``graph._graph`` -> its device index; ``ret`` without
    requires_grad: the output of the Function carries the gradient)."""
    g = graph._graph.get_immutable_gidx(weight.device)
    ret = th.zeros((weight.size(1), weight.size(2)), dtype=weight.dtype, device=weight.device)
    return RgcnFirstLayer.apply(g, weight, norm, ret)


class RgcnSecondLayer(th.autograd.Function):
    """tensor.py:468-490; also returns the weight gradient the C entry fills."""

    @staticmethod
    def forward(ctx, graph, x, weight, norm, ret):
        ctx.backward_cache = graph, weight, norm, x
        K.rgcn_layer1(graph, x, weight, norm, ret)
        return ret

    @staticmethod
    def backward(ctx, gradout):
        graph, weight, norm, x = ctx.backward_cache
        grad_x = th.zeros_like(x)
        grad_weight = th.zeros_like(weight)
        K.rgcn_layer1_backward(graph, x, weight, norm, gradout.contiguous(), grad_x, grad_weight)
        return None, grad_x, grad_weight, None, None


def rgcn_layer1(graph, x, weight, norm):
    """tensor.py:492-495."""
    g = graph._graph.get_immutable_gidx(x.device)
    ret = th.zeros((graph.number_of_nodes(), weight.size(2)), dtype=weight.dtype,
                   device=weight.device)
    return RgcnSecondLayer.apply(g, x, weight, norm, ret)


def _typed_graph(n, m, R, seed, hub):
    rng = np.random.default_rng(seed)
    if hub:
        src, dst, n = powerlaw(n, m, seed=seed)
    else:
        src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    src[: m // 10] = src[0]                      # repeated (source, relation) pairs
    et = rng.integers(0, R, len(src))
    norm = rng.uniform(0.1, 1.0, (len(src), 1)).astype(np.float32)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges_with_type(src, dst, et)          # graph.py:1229 (the hack)
    return g, src, dst, et, norm, n


@pytest.mark.parametrize("F,hub", [(16, False), (7, True)])
def test_reference_order_layer0_vs_oracle(F, hub):
    R = 3
    g, src, dst, et, norm, n = _typed_graph(700, 9000, R, seed=F, hub=hub)
    rng = np.random.default_rng(F + 1)
    w = rng.standard_normal((R, n, F)).astype(np.float32)
    go = rng.standard_normal((n, F)).astype(np.float32)
    wd = th.from_numpy(w).to(DEV).requires_grad_()
    nd = th.from_numpy(norm).to(DEV)
    out = rgcn_layer0(g, wd, nd)
    (gw,) = th.autograd.grad(out, (wd,), th.from_numpy(go).to(DEV))
    _close(out.detach().cpu(), O.hack_rgcn_layer0(src, dst, et, n, w, norm),
           O.hack_rgcn_layer0(src, dst, et, n, np.abs(w), norm), "layer0")
    _close(gw.cpu(), O.hack_rgcn_layer0_backward(src, dst, et, n, go, norm, R, accumulate=True),
           O.hack_rgcn_layer0_backward(src, dst, et, n, np.abs(go), norm, R, accumulate=True),
           "layer0 backward")


@pytest.mark.parametrize("K_in,X,prepare,hub", [(16, 16, 0, False), (20, 5, 0, True),
                                               (64, 64, 3, True), (64, 64, 4, False)])
def test_reference_order_layer1_vs_oracle(K_in, X, prepare, hub):
    """prepare 0: stateless; 3: the prepared relation-expanded CSRs; 4: the fused
    aggregate-then-transform kernels -- all reached through the 5- and 7-argument
    entries, the prepared state found on the graph."""
    R = 4
    g, src, dst, et, norm, n = _typed_graph(900, 12000, R, seed=K_in + X, hub=hub)
    rng = np.random.default_rng(X)
    h = rng.standard_normal((n, K_in)).astype(np.float32)
    w = (rng.standard_normal((R, K_in, X)) / 4).astype(np.float32)
    go = rng.standard_normal((n, X)).astype(np.float32)
    nd = th.from_numpy(norm).to(DEV)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    assert gidx.etypes is not None and gidx.etypes.dtype == th.int32
    gidx.__dict__.pop("_rgcn_state", None)
    if prepare:
        K.rgcn_prepare(gidx, nd, R, layers=prepare)  # the graph's own relation ids
    hd = th.from_numpy(h).to(DEV).requires_grad_()
    wd = th.from_numpy(w).to(DEV).requires_grad_()
    out = rgcn_layer1(g, hd, wd, nd)
    gh, gw = th.autograd.grad(out, (hd, wd), th.from_numpy(go).to(DEV))
    gidx.__dict__.pop("_rgcn_state", None)
    _close(out.detach().cpu(), O.hack_rgcn_layer1(src, dst, et, n, h, w, norm),
           O.hack_rgcn_layer1(src, dst, et, n, np.abs(h), np.abs(w), norm), "layer1")
    gh_ref, gw_ref = O.hack_rgcn_layer1_backward(src, dst, et, n, h, w, norm, go)
    gh_mass, gw_mass = O.hack_rgcn_layer1_backward(src, dst, et, n, np.abs(h), np.abs(w), norm,
                                                   np.abs(go))
    _close(gh.cpu(), gh_ref, gh_mass, "grad_hidden")
    _close(gw.cpu(), gw_ref, gw_mass, "grad_weight")


def test_raw_ctypes_argument_lists():
    """The four entries called directly through ctypes with exactly the reference's
    argument lists (plus the stream), the relation ids only in the graph struct."""
    R, F = 3, 16
    g, src, dst, et, norm, n = _typed_graph(400, 5000, R, seed=2, hub=False)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    gs = gidx.cstruct()
    gs.etypes = gidx.etypes.data_ptr()
    L = _ffi.lib()
    arr = K._arr
    stream = th.cuda.current_stream().cuda_stream
    nd = th.from_numpy(norm).to(DEV)
    w0 = th.randn(R, n, F, device=DEV)
    ret0 = th.zeros(n, F, device=DEV)
    _ffi.check_call(L.DGLMIRgcnLayer0(ctypes.byref(gs), arr(w0, "w"), arr(nd, "n"),
                                      arr(ret0, "r"), stream))
    go0 = th.randn(n, F, device=DEV)
    gw0 = th.zeros(R, n, F, device=DEV)
    _ffi.check_call(L.DGLMIRgcnLayer0Backward(ctypes.byref(gs), arr(go0, "g"), arr(nd, "n"),
                                              arr(gw0, "gw"), stream))
    h = th.randn(n, F, device=DEV)
    w1 = th.randn(R, F, 8, device=DEV)
    ret1 = th.zeros(n, 8, device=DEV)
    _ffi.check_call(L.DGLMIRgcnLayer1(ctypes.byref(gs), arr(h, "h"), arr(w1, "w"), arr(nd, "n"),
                                      arr(ret1, "r"), stream))
    go1 = th.randn(n, 8, device=DEV)
    gh1, gw1 = th.zeros_like(h), th.zeros_like(w1)
    _ffi.check_call(L.DGLMIRgcnLayer1Backward(ctypes.byref(gs), arr(h, "h"), arr(w1, "w"),
                                              arr(nd, "n"), arr(go1, "g"), arr(gh1, "gh"),
                                              arr(gw1, "gw"), stream))
    th.cuda.synchronize()
    nn_ = norm.astype(np.float32)
    _close(ret0.cpu(), O.hack_rgcn_layer0(src, dst, et, n, w0.cpu().numpy(), nn_),
           O.hack_rgcn_layer0(src, dst, et, n, np.abs(w0.cpu().numpy()), nn_), "layer0")
    _close(ret1.cpu(), O.hack_rgcn_layer1(src, dst, et, n, h.cpu().numpy(), w1.cpu().numpy(), nn_),
           O.hack_rgcn_layer1(src, dst, et, n, np.abs(h.cpu().numpy()), np.abs(w1.cpu().numpy()),
                              nn_), "layer1")
    ghr, gwr = O.hack_rgcn_layer1_backward(src, dst, et, n, h.cpu().numpy(), w1.cpu().numpy(), nn_,
                                           go1.cpu().numpy())
    ghm, gwm = O.hack_rgcn_layer1_backward(src, dst, et, n, np.abs(h.cpu().numpy()),
                                           np.abs(w1.cpu().numpy()), nn_,
                                           np.abs(go1.cpu().numpy()))
    _close(gh1.cpu(), ghr, ghm, "grad_hidden")
    _close(gw1.cpu(), gwr, gwm, "grad_weight")
    # an untyped graph struct is refused, not read out of bounds
    gs.etypes = None
    assert L.DGLMIRgcnLayer0(ctypes.byref(gs), arr(w0, "w"), arr(nd, "n"), arr(ret0, "r"),
                             stream) != 0
    assert "edge types" in _ffi.last_error()


def test_rebuild_keeps_one_state():
    """A new set of relation ids releases the graph's old prepared state before the
    new one is allocated (two C5-size states would hold ~4 GB outside the caching
    allocator)."""
    import gc
    R = 4
    g, src, dst, et, norm, n = _typed_graph(3000, 40000, R, seed=5, hub=False)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    nd = th.from_numpy(norm).to(DEV)
    gc.collect()
    before = K.RgcnState.live
    st1 = K.rgcn_prepare(gidx, nd, R, layers=6)
    assert K.RgcnState.live == before + 1
    et2 = ((gidx.etypes + 1) % R).contiguous()
    st2 = K.rgcn_prepare(gidx, nd, R, layers=6, etypes=et2)
    assert K.RgcnState.live == before + 1 and not st1._fin.alive and st2._fin.alive
    gidx.__dict__.pop("_rgcn_state").release()
    assert K.RgcnState.live == before
