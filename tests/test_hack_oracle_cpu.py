"""Pins the oracle's restatement of the hack's GPU-only kernels (``oracle/hack_ref.c``)
before the GPU tests trust it.

* Fused GAT (``binary_reduce_impl.cu:47-213``): the reference's own check
  (``examples/pytorch/gat/fused_gat_unit_test.py:37-73``) compares the fused kernel
  with the builtin composition u_add_v -> leaky_relu -> exp -> copy_e sum -> e_div_v ->
  u_mul_e sum, and el / er gradients by autograd.  Restated here: the forward against
  that composition on the oracle's builtin kernels (``dgl_ref.c``), every gradient
  against torch fp64 autograd of the same composition, on the unit test's own graph
  (every node -> 0 and -> 1) and a random one.
* R-GCN (``:913-1245``): the hack's layers replace upstream RelGraphConv's per-edge
  message ``bmm(h[src], W[type]) * norm`` (layer 1) and ``W[type, src] * norm``
  (layer 0, embedding input), summed per destination
  (``examples/pytorch/rgcn/egl_entity_classify.py:98-116``); restated in fp64 with
  autograd gradients.  The layer-0 backward's store (``:1004``) is checked to equal the
  exact gradient when no (source, relation) pair repeats and to keep only the last
  edge's term when one does.
* ``GetCsrSortedByEdgeType`` (``src/graph/graph.cc:690-746``): a spelled-out known
  answer.
"""
import numpy as np
import pytest
import torch as th

from oracle import oracle as O


def _unit_test_graph(n):
    # fused_gat_unit_test.py:17-20: every node -> 0, then every node -> 1
    src = np.concatenate([np.arange(n), np.arange(n)])
    dst = np.concatenate([np.zeros(n, np.int64), np.ones(n, np.int64)])
    return src, dst


def _random_graph(n, m, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, n, m), rng.integers(0, n, m)


def _composition_f64(src, dst, n, ft, el, er, slope):
    """The unit test's expected_output() as fp64 torch ops (autograd-able)."""
    s, d = th.from_numpy(src), th.from_numpy(dst)
    e = el[s] + er[d]                                   # u_add_v, (E, H, 1)
    e = th.nn.functional.leaky_relu(e, slope).exp()
    den = th.zeros(n, *e.shape[1:], dtype=e.dtype).index_add(0, d, e)   # copy_e sum
    a = e / den[d]                                      # e_div_v
    return th.zeros(n, *ft.shape[1:], dtype=ft.dtype).index_add(0, d, ft[s] * a)


def _composition_oracle(src, dst, n, ft, el, er, slope):
    """The same composition on the oracle's builtin kernels (fp32, dgl_ref.c)."""
    g = O.RefGraph(src, dst, n)
    e = O.binary_reduce("none", "add", g, O.SRC, O.DST, el, er, g.m)
    e = np.where(e > 0, e, slope * e).astype(np.float32)
    e = np.exp(e).astype(np.float32)
    den = O.copy_reduce("sum", g, O.EDGE, e, n)
    a = O.binary_reduce("none", "div", g, O.EDGE, O.DST, e, den, g.m)
    return O.binary_reduce("sum", "mul", g, O.SRC, O.EDGE, ft, a, n)


@pytest.mark.parametrize("graph", ["unit_test", "random"])
def test_fused_gat_oracle_matches_builtin_composition(graph):
    H, D, slope = 4, 8, 0.2
    if graph == "unit_test":
        n = 64
        src, dst = _unit_test_graph(n)
    else:
        n = 300
        src, dst = _random_graph(n, 4000, seed=3)
    rng = np.random.default_rng(11)
    ft = rng.standard_normal((n, H, D)).astype(np.float32)
    el = rng.random((n, H, 1)).astype(np.float32)   # th.rand, as the unit test
    er = rng.random((n, H, 1)).astype(np.float32)
    exp, s, ret = O.hack_fused_gat(src, dst, n, ft, el, er, slope)
    comp = _composition_oracle(src, dst, n, ft, el, er, slope)
    np.testing.assert_allclose(ret, comp, rtol=1e-5, atol=1e-6)
    # the unit test's grads (el, er) and the feature gradient, fp64 autograd
    ftd, eld, erd = (th.from_numpy(x).double().requires_grad_() for x in (ft, el, er))
    ref = _composition_f64(src, dst, n, ftd, eld, erd, slope)
    np.testing.assert_allclose(ret, ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    go = rng.standard_normal(ret.shape).astype(np.float32)
    gref = th.autograd.grad(ref, (ftd, eld, erd), th.from_numpy(go).double())
    gfs, gel, ger = O.hack_fused_gat_backward(src, dst, n, ft, el, er, s, exp, ret, go, slope)
    for a, b, name in zip((gfs, gel, ger), gref, ("feat_src", "el", "er")):
        np.testing.assert_allclose(a, b.numpy(), rtol=1e-4, atol=1e-5, err_msg=name)
    # the forward's state: exp per edge id, sum per destination
    e = el[src, :, 0] + er[dst, :, 0]
    np.testing.assert_allclose(exp, np.exp(np.where(e > 0, e, slope * e)), rtol=1e-6)
    np.testing.assert_allclose(s, np.bincount(np.repeat(dst, H) * H + np.tile(np.arange(H), len(dst)),
                                              exp.reshape(-1), minlength=n * H).reshape(n, H),
                               rtol=1e-5)


def _rgcn_graph(n, m, R, seed, repeat_pairs):
    rng = np.random.default_rng(seed)
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    et = rng.integers(0, R, m)
    if repeat_pairs:
        src[: m // 10] = src[0]
        et[: m // 10] = et[0]
    norm = rng.uniform(0.1, 1.0, (m, 1)).astype(np.float32)
    return src, dst, et, norm


def test_rgcn_layer1_oracle_matches_per_edge_bmm():
    n, m, R, Y, X = 200, 3000, 3, 12, 10
    src, dst, et, norm = _rgcn_graph(n, m, R, seed=5, repeat_pairs=True)
    rng = np.random.default_rng(6)
    h = rng.standard_normal((n, Y)).astype(np.float32)
    w = rng.standard_normal((R, Y, X)).astype(np.float32)
    out = O.hack_rgcn_layer1(src, dst, et, n, h, w, norm)
    hd, wd = th.from_numpy(h).double().requires_grad_(), th.from_numpy(w).double().requires_grad_()
    s, d, t = th.from_numpy(src), th.from_numpy(dst), th.from_numpy(et)
    msg = th.bmm(hd[s].unsqueeze(1), wd[t]).squeeze(1) * th.from_numpy(norm).double()
    ref = th.zeros(n, X, dtype=th.float64).index_add(0, d, msg)
    np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-5, atol=1e-5)
    go = rng.standard_normal((n, X)).astype(np.float32)
    gh, gw = O.hack_rgcn_layer1_backward(src, dst, et, n, h, w, norm, go)
    gh_ref, gw_ref = th.autograd.grad(ref, (hd, wd), th.from_numpy(go).double())
    np.testing.assert_allclose(gh, gh_ref.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(gw, gw_ref.numpy(), rtol=1e-5, atol=1e-4)


def test_rgcn_layer0_oracle_and_the_reference_store():
    n, m, R, F = 150, 2000, 4, 9
    rng = np.random.default_rng(7)
    w = rng.standard_normal((R, n, F)).astype(np.float32)
    for repeat in (False, True):
        src, dst, et, norm = _rgcn_graph(n, m, R, seed=8, repeat_pairs=repeat)
        if not repeat:
            # one edge per (source, relation) pair: the reference's store is exact
            key = np.arange(m) % (n * R)
            src, et = key % n, key // n
            src, dst, et, norm = src[: n * R], dst[: n * R], et[: n * R], norm[: n * R]
        out = O.hack_rgcn_layer0(src, dst, et, n, w, norm)
        wd = th.from_numpy(w).double().requires_grad_()
        s, d, t = th.from_numpy(src), th.from_numpy(dst), th.from_numpy(et)
        ref = th.zeros(n, F, dtype=th.float64).index_add(0, d, wd[t, s] * th.from_numpy(norm).double())
        np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-5, atol=1e-5)
        go = rng.standard_normal((n, F)).astype(np.float32)
        (gw_ref,) = th.autograd.grad(ref, (wd,), th.from_numpy(go).double())
        exact = O.hack_rgcn_layer0_backward(src, dst, et, n, go, norm, R, accumulate=True)
        stored = O.hack_rgcn_layer0_backward(src, dst, et, n, go, norm, R, accumulate=False)
        np.testing.assert_allclose(exact, gw_ref.numpy(), rtol=1e-5, atol=1e-5)
        if not repeat:
            np.testing.assert_array_equal(stored, exact)
        else:
            # the repeated pair (src[0], et[0]) keeps only its last out-edge's term in
            # type-sorted out-CSR order (= the largest edge id of that type)
            u, t = src[0], et[0]
            eids = np.nonzero((src == u) & (et == t))[0]
            last = eids.max()
            np.testing.assert_allclose(stored[t, u], go[dst[last]] * norm[last, 0], rtol=1e-6)
            assert not np.allclose(stored[t, u], exact[t, u])


def test_sort_rows_by_type_known_answer():
    # 4 nodes; edges in id order: (0->1,t2) (0->2,t0) (3->1,t1) (0->3,t0) (2->1,t0)
    src = np.array([0, 0, 3, 0, 2])
    dst = np.array([1, 2, 1, 3, 1])
    et = np.array([2, 0, 1, 0, 0])
    ptr, ids, eids, types = O.csr_sorted_by_edge_type(src, dst, et, 4, 3, transpose=True)
    assert ptr.tolist() == [0, 3, 3, 4, 5]
    assert ids.tolist() == [2, 3, 1, 1, 1]       # row 0: eids 1 (t0), 3 (t0), 0 (t2)
    assert eids.tolist() == [1, 3, 0, 4, 2]
    assert types.tolist() == [0, 0, 2, 0, 1]
    ptr, ids, eids, types = O.csr_sorted_by_edge_type(src, dst, et, 4, 3, transpose=False)
    assert ptr.tolist() == [0, 0, 3, 4, 5]
    assert ids.tolist() == [2, 3, 0, 0, 0]       # row 1: eids 4 (t0), 2 (t1), 0 (t2)
    assert eids.tolist() == [4, 2, 0, 1, 3]
    assert types.tolist() == [0, 1, 2, 0, 0]
    with pytest.raises(ValueError):
        O.csr_sorted_by_edge_type(src, dst, et, 4, 2, transpose=True)
