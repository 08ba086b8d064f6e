"""The hack's fused-GAT PackedFuncs in the reference's own argument order
(``DGLMIFusedGatKernel`` / ``DGLMIKernelBackwardFusedGat``; reference
``src/kernel/binary_reduce.cc:380-396, 529-549``), called through ctypes by a
restatement of the reference's caller (``python/dgl/backend/pytorch/tensor.py:
383-420``: ``exp`` = (E, H, 1), ``s`` = empty_like(el), ``ret`` =
empty_like(feat_src), zero-filled gradients), against the dense fp64
restatement of GAT attention (test_fused_gat_gpu.dense_gat)."""
import numpy as np
import pytest
import torch as th

import dgl
import dgl.backend as B
from dgl import kernel as K
from graphs import powerlaw
from test_fused_gat_gpu import dense_gat

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class RefFusedGat(th.autograd.Function):
    """tensor.py:383-413, with the kernel calls bound to libdglmi in the same order."""

    @staticmethod
    def forward(ctx, graph, feat_src, el, er, s, exp, ret, slope):
        ctx.backward_cache = graph, feat_src, el, er, s, exp, ret, slope
        K.fused_gat_kernel(graph, feat_src, el, er, s, exp, ret, slope)
        return ret

    @staticmethod
    def backward(ctx, gradout):
        graph, feat_src, el, er, s, exp, ret, slope = ctx.backward_cache
        grad_el = th.zeros_like(el)
        grad_er = th.zeros_like(er)
        grad_feat_src = th.zeros_like(feat_src)
        K.backward_fused_gat(graph, feat_src, el, er, s, exp, ret, gradout.contiguous(),
                             grad_feat_src, grad_el, grad_er, slope)
        return None, grad_feat_src, grad_el, grad_er, None, None, None, None


def ref_fused_gat(graph, feat_src, el, er, slope):
    """tensor.py:415-420."""
    g = graph._graph.get_immutable_gidx(th.device(DEV))
    exp = el.new_empty([g.number_of_edges()] + list(el.size()[1:]))
    s = th.empty_like(el)
    ret = th.empty_like(feat_src)
    return RefFusedGat.apply(g, feat_src, el, er, s, exp, ret, slope), s, exp


def _check(src, dst, n, H, D, seed):
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gen = th.Generator(device=DEV).manual_seed(seed)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    er = (3 * th.randn(n, H, 1, device=DEV, generator=gen)).requires_grad_()
    out, s, exp = ref_fused_gat(g, ft, el, er, 0.2)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gf = th.autograd.grad(out, (ft, el, er), go)
    fd, eld, erd = (t.detach().double().requires_grad_() for t in (ft, el, er))
    ref = dense_gat(src, dst, n, fd, eld, erd, 0.2)
    gr = th.autograd.grad(ref, (fd, eld, erd), go.double())
    assert th.allclose(out.double(), ref, rtol=1e-4, atol=1e-4)
    for a, b, name in zip(gf, gr, ("ft", "el", "er")):
        assert th.allclose(a.double(), b, rtol=1e-3, atol=1e-3), name
    zero = th.from_numpy(np.bincount(dst, minlength=n) == 0).to(DEV)
    assert (out[zero] == 0).all()
    return g, (ft, el, er), out, gf, go


@pytest.mark.parametrize("H,D", [(8, 8), (3, 16)])
def test_reference_order_matches_dense_and_native(H, D):
    # E >= N: exp's first N*H floats carry the running max -- the same kernels as the
    # native entry, so the results are bit-identical to dgl.backend.fused_gat
    src, dst, n = powerlaw(20000, 300000, seed=17)
    g, (ft, el, er), out, gf, go = _check(src, dst, n, H, D, seed=4)
    # exp also holds the slope aggregates when E * H >= round_up(N H, 4) + N H (D + 1)
    # (dglmi.h); the native entry then keeps them too, else neither does
    holds = len(src) * H >= ((n * H + 3) // 4) * 4 + n * H * (D + 1)
    import os
    os.environ["DGLMI_GAT_SLOPES"] = "1" if holds else "0"
    try:
        nat = B.fused_gat(g, ft, el, er, 0.2)
    finally:
        os.environ.pop("DGLMI_GAT_SLOPES")
    assert th.equal(nat, out)
    gn = th.autograd.grad(nat, (ft, el, er), go)
    for a, b in zip(gn, gf):
        assert th.equal(a, b)


def test_reference_order_fewer_edges_than_nodes():
    # E < N (most nodes isolated): exp is too small for the max, so s keeps the
    # log-sum-exp and the backward's attention is exp(logit - lse)
    rng = np.random.default_rng(5)
    n, m = 50000, 20000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, 2000, m)  # 2000 destinations, the rest have no in-edge
    _check(src, dst, n, 8, 8, seed=6)


def test_reference_order_column_blocks(monkeypatch):
    monkeypatch.setenv("DGLMI_GAT_BLOCKS", "4")
    src, dst, n = powerlaw(20000, 300000, seed=19)
    _check(src, dst, n, 8, 8, seed=8)


def test_reference_order_rejects_wrong_state_shapes():
    src, dst, n = powerlaw(2000, 20000, seed=3)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(th.device(DEV))
    ft = th.randn(n, 8, 8, device=DEV)
    el = th.randn(n, 8, 1, device=DEV)
    ret = th.empty_like(ft)
    with pytest.raises(dgl.DGLError, match="exp must be"):
        K.fused_gat_kernel(gidx, ft, el, el, th.empty_like(el), th.empty(10, 8, 1, device=DEV),
                           ret, 0.2)
    with pytest.raises(dgl.DGLError, match="sum must be"):
        K.fused_gat_kernel(gidx, ft, el, el, th.empty(n - 1, 8, device=DEV),
                           th.empty(len(src), 8, 1, device=DEV), ret, 0.2)
