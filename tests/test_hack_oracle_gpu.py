"""The hack's GPU-only entry points through the C ABI against the oracle's
restatement of the hack's own CUDA kernels (``oracle/hack_ref.c``, pinned by
``tests/test_hack_oracle_cpu.py``): the reference-order fused GAT
(``DGLMIFusedGatKernel`` / ``DGLMIKernelBackwardFusedGat``,
``binary_reduce.cc:380-396, 529-549``) and ``DGLMIRgcnLayer0/1[Backward]``
(``:398-450``), stateless, with prepared per-graph state, and on the fused layer-1
kernels.

Tolerance: both sides sum in fp32, in different orders (the oracle in the hack's
per-thread order, the product in chunked load-balanced order, the GAT with a running
max), so every check bounds |product - oracle| by 1e-5 + 2e-5 * (the sum of the
absolute terms), evaluated in fp64.  The layer-0 backward is compared with the exact
sum (the reference's store keeps only the last edge of a repeated (source, relation)
pair, ``binary_reduce_impl.cu:1004``)."""
import numpy as np
import pytest
import torch as th

import dgl
from dgl import kernel as K
from graphs import powerlaw
from oracle import oracle as O
from test_fused_gat_refabi_gpu import ref_fused_gat

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _close(got, want, mass, what):
    got = np.asarray(got, np.float64)
    bound = 1e-5 + 2e-5 * np.asarray(mass, np.float64)
    err = np.abs(got - np.asarray(want, np.float64))
    assert (err <= bound).all(), "%s: worst err/bound %.3g" % (what, float((err / bound).max()))


def _graphs():
    n = 96
    us = (np.concatenate([np.arange(n), np.arange(n)]),
          np.concatenate([np.zeros(n, np.int64), np.ones(n, np.int64)]), n)
    rng = np.random.default_rng(21)
    rnd = (rng.integers(0, 500, 6000), rng.integers(0, 500, 6000), 500)
    src, dst, pn = powerlaw(800, 12000, seed=23)
    return {"unit_test": us, "random": rnd, "powerlaw": (src, dst, pn)}


@pytest.mark.parametrize("name", ["unit_test", "random", "powerlaw"])
@pytest.mark.parametrize("H,D", [(8, 8), (3, 16)])
def test_fused_gat_reference_order_vs_oracle(name, H, D):
    src, dst, n = _graphs()[name]
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gen = th.Generator(device=DEV).manual_seed(H * 100 + D)
    ft = th.randn(n, H, D, device=DEV, generator=gen).requires_grad_()
    el = th.rand(n, H, 1, device=DEV, generator=gen).requires_grad_()
    er = th.rand(n, H, 1, device=DEV, generator=gen).requires_grad_()
    out, _, _ = ref_fused_gat(g, ft, el, er, 0.2)
    go = th.randn(out.shape, device=DEV, generator=gen)
    gft, gel, ger = th.autograd.grad(out, (ft, el, er), go)
    f, l, r, gon = (t.detach().cpu().numpy() for t in (ft, el, er, go))
    exp, s, ret = O.hack_fused_gat(src, dst, n, f, l, r, 0.2)
    ofs, oel, oer = O.hack_fused_gat_backward(src, dst, n, f, l, r, s, exp, ret, gon, 0.2)
    # absolute masses of the sums (attention weights are in [0, 1])
    sd, dd = th.from_numpy(src), th.from_numpy(dst)
    fabs = th.from_numpy(np.abs(f)).double()
    out_mass = th.zeros(n, H, D, dtype=th.float64).index_add(0, dd, fabs[sd])
    goabs = th.from_numpy(np.abs(gon)).double()
    gfs_mass = th.zeros(n, H, D, dtype=th.float64).index_add(0, sd, goabs[dd])
    term = (goabs[dd] * (fabs[sd] + th.from_numpy(np.abs(ret)).double()[dd])).sum(-1)
    gel_mass = th.zeros(n, H, dtype=th.float64).index_add(0, sd, term)
    ger_mass = th.zeros(n, H, dtype=th.float64).index_add(0, dd, term)
    _close(out.detach().cpu(), ret, out_mass, "ret")
    _close(gft.cpu(), ofs, gfs_mass, "grad_feat_src")
    _close(gel.cpu().reshape(n, H), oel.reshape(n, H), gel_mass, "grad_el")
    _close(ger.cpu().reshape(n, H), oer.reshape(n, H), ger_mass, "grad_er")


def _rgcn_case(n, m, R, seed, hub):
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
    g.add_edges(src, dst)
    gidx = g._graph.get_immutable_gidx(DEV)
    return src, dst, et, norm, n, gidx


@pytest.mark.parametrize("F,hub", [(16, False), (7, True)])
def test_rgcn_layer0_vs_oracle(F, hub):
    R = 3
    src, dst, et, norm, n, gidx = _rgcn_case(700, 9000, R, seed=F, hub=hub)
    rng = np.random.default_rng(F + 1)
    w = rng.standard_normal((R, n, F)).astype(np.float32)
    go = rng.standard_normal((n, F)).astype(np.float32)
    et32, nd = th.from_numpy(et).int().to(DEV), th.from_numpy(norm).to(DEV)
    ret = th.full((n, F), float("nan"), device=DEV)
    K.rgcn_layer0(gidx, th.from_numpy(w).to(DEV), nd, ret, etypes=et32)
    gw = th.full((R, n, F), float("nan"), device=DEV)
    K.rgcn_layer0_backward(gidx, th.from_numpy(go).to(DEV), nd, gw, etypes=et32)
    oref = O.hack_rgcn_layer0(src, dst, et, n, w, norm)
    omass = O.hack_rgcn_layer0(src, dst, et, n, np.abs(w), norm)
    _close(ret.cpu(), oref, omass, "layer0")
    gref = O.hack_rgcn_layer0_backward(src, dst, et, n, go, norm, R, accumulate=True)
    gmass = O.hack_rgcn_layer0_backward(src, dst, et, n, np.abs(go), norm, R, accumulate=True)
    _close(gw.cpu(), gref, gmass, "layer0 backward")


@pytest.mark.parametrize("K_in,X,prepare,hub", [(16, 16, 0, False), (20, 5, 0, True),
                                               (64, 64, 3, False), (64, 48, 4, True),
                                               (64, 100, 4, False)])
def test_rgcn_layer1_vs_oracle(K_in, X, prepare, hub):
    """prepare 0: stateless entries; 3: prepared relation-expanded CSRs; 4: the fused
    aggregate-then-transform kernels (64-wide inputs, outputs <= 128)."""
    R = 4
    src, dst, et, norm, n, gidx = _rgcn_case(900, 12000, R, seed=K_in + X, hub=hub)
    rng = np.random.default_rng(X)
    h = rng.standard_normal((n, K_in)).astype(np.float32)
    w = (rng.standard_normal((R, K_in, X)) / 4).astype(np.float32)
    go = rng.standard_normal((n, X)).astype(np.float32)
    et32, nd = th.from_numpy(et).int().to(DEV), th.from_numpy(norm).to(DEV)
    gidx.__dict__.pop("_rgcn_state", None)
    if prepare:
        K.rgcn_prepare(gidx, nd, R, layers=prepare, etypes=et32)
    hd, wd, god = (th.from_numpy(a).to(DEV) for a in (h, w, go))
    ret = th.full((n, X), float("nan"), device=DEV)
    K.rgcn_layer1(gidx, hd, wd, nd, ret, etypes=et32)
    gh = th.full((n, K_in), float("nan"), device=DEV)
    gw = th.full((R, K_in, X), float("nan"), device=DEV)
    K.rgcn_layer1_backward(gidx, hd, wd, nd, god, gh, gw, etypes=et32)
    gidx.__dict__.pop("_rgcn_state", None)
    oref = O.hack_rgcn_layer1(src, dst, et, n, h, w, norm)
    omass = O.hack_rgcn_layer1(src, dst, et, n, np.abs(h), np.abs(w), norm)
    _close(ret.cpu(), oref, omass, "layer1")
    gh_ref, gw_ref = O.hack_rgcn_layer1_backward(src, dst, et, n, h, w, norm, go)
    gh_mass, gw_mass = O.hack_rgcn_layer1_backward(src, dst, et, n, np.abs(h), np.abs(w), norm,
                                                   np.abs(go))
    _close(gh.cpu(), gh_ref, gh_mass, "grad_hidden")
    _close(gw.cpu(), gw_ref, gw_mass, "grad_weight")
