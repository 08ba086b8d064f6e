"""The CPU oracle pinned against the reference's own known answers (no GPU)."""
import itertools
import json
import os

import numpy as np
import pytest
import torch as th

from oracle import oracle as O
from oracle import udf_ref as U
from graphs import CODE, binary_case_features, er_graph, g20

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "spmat_kat.json")))


def _eq(a, b):
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def test_coo_to_csr_kat():
    # tests/cpp/test_spmat.cc:358-372 (unsorted COO -> CSR1 / CSR2)
    for coo, csr in (("COO1", "CSR1"), ("COO2", "CSR2")):
        p, i, d = O.coo_to_csr(KAT["num_rows"], KAT[coo]["row"], KAT[coo]["col"])
        _eq(p, KAT[csr]["indptr"]); _eq(i, KAT[csr]["indices"]); _eq(d, KAT[csr]["data"])


def test_coo_to_csr_sorted_kat():
    # COOSort(row) / COOSort(row, col) then COOToCSR (test_spmat.cc:374-416)
    row = np.array(KAT["COO3"]["row"]); col = np.array(KAT["COO3"]["col"])
    perm = np.argsort(row, kind="stable")
    p, i, d = O.coo_to_csr(4, row[perm], col[perm], perm)
    _eq(p, KAT["SR_CSR3"]["indptr"]); _eq(i, KAT["SR_CSR3"]["indices"]); _eq(d, KAT["SR_CSR3"]["data"])
    perm = np.lexsort((col, row))
    p, i, d = O.coo_to_csr(4, row[perm], col[perm], perm)
    _eq(p, KAT["SRC_CSR3"]["indptr"]); _eq(i, KAT["SRC_CSR3"]["indices"]); _eq(d, KAT["SRC_CSR3"]["data"])


def test_csr_transpose_kat():
    c = KAT["CSR2"]
    p, i, d = O.csr_transpose(4, 5, c["indptr"], c["indices"], c["data"])
    t = KAT["CSR2_T"]
    _eq(p, t["indptr"]); _eq(i, t["indices"]); _eq(d, t["data"])


def test_csr_to_coo_kat():
    rows = O.csr_to_coo_rows(4, KAT["CSR2"]["indptr"])
    _eq(rows, KAT["CSR2_TO_COO"]["row"])


def test_infer_shape():
    f = lambda op, a, b: O.infer_binary_feature_shape(op, np.zeros(a, np.float32), np.zeros(b, np.float32))
    assert f("add", (3, 5, 3, 4), (3, 3, 1)) == (5, 3, 4)
    assert f("mul", (3, 4), (3, 5, 3, 4)) == (5, 3, 4)
    assert f("dot", (3, 5, 1, 10), (3, 5, 3, 10)) == (5, 3, 10)
    with pytest.raises(ValueError):
        f("add", (3, 5), (3, 4))


def _udf_compare(src, dst, n, lhs, rhs, op, red, bc, partial=False):
    m = len(src)
    d = binary_case_features(n, m, lhs, rhs, op, bc)
    g = O.RefGraph(src, dst, n)
    out = O.binary_reduce(red, op, g, CODE[lhs], CODE[rhs], d[lhs], d[rhs], n)
    res, grads = U.update_all(src, dst, n, lhs, rhs, op, red,
                              {k: th.from_numpy(x) for k, x in d.items()})
    _, gl, gr = O.binary_reduce(red, op, g, CODE[lhs], CODE[rhs], d[lhs], d[rhs], n,
                                grad_out=np.ones_like(out))
    tol = 1e-2 if red == "prod" else 1e-4
    np.testing.assert_allclose(out, res.numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(gl, grads[lhs].numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(gr, grads[rhs].numpy(), rtol=tol, atol=tol)


@pytest.mark.parametrize("lhs,rhs", [(a, b) for a, b in itertools.product("uve", "uve") if a != b])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "dot"])
def test_oracle_vs_udf_g20(lhs, rhs, op):
    """test_kernel.py:200-362 methodology: builtin (oracle) vs UDF/degree bucketing."""
    src, dst, n = g20()
    for red in ["sum", "max", "min", "prod", "mean"]:
        for bc in ["none", lhs, rhs]:
            _udf_compare(src, dst, n, lhs, rhs, op, red, bc)


@pytest.mark.parametrize("red", ["sum", "max", "mean"])
def test_oracle_copy_src_er(red):
    """test_kernel.py:77-136: copy_src x {sum,max,mean} on ER(100, 0.1) + self-loops."""
    src, dst, n = er_graph()
    x = np.random.RandomState(31).uniform(-1, 1, (n, 5, 3, 4)).astype(np.float32)
    g = O.RefGraph(src, dst, n)
    out, gx = O.copy_reduce(red, g, O.SRC, x, n, grad_out=np.ones((n, 5, 3, 4), np.float32))
    res, grads = U.update_all(src, dst, n, "u", None, None, red, {"u": th.from_numpy(x)})
    np.testing.assert_allclose(out, res.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gx, grads["u"].numpy(), rtol=1e-4, atol=1e-4)


def test_oracle_threads_agree():
    """The multi-threaded (omp atomic) reference order agrees with the serial one."""
    src, dst, n = er_graph(300, 0.05, seed=3)
    x = np.random.RandomState(1).uniform(-1, 1, (n, 16)).astype(np.float32)
    g = O.RefGraph(src, dst, n)
    a = O.copy_reduce("sum", g, O.SRC, x, n, nthreads=1)
    b = O.copy_reduce("sum", g, O.SRC, x, n, nthreads=4)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    out, gi = O.copy_reduce("max", g, O.SRC, x, n, nthreads=1), None
    np.testing.assert_array_equal(out, O.copy_reduce("max", g, O.SRC, x, n, nthreads=4))


def test_zero_degree_identity():
    """Builtin reducers leave the identity on zero-in-degree nodes (binary_reduce_impl.h:62)."""
    src, dst, n = np.array([0, 1]), np.array([1, 1]), 3
    g = O.RefGraph(src, dst, n)
    x = np.ones((3, 2), np.float32)
    assert (O.copy_reduce("max", g, O.SRC, x, n)[0] == np.finfo(np.float32).min).all()
    assert (O.copy_reduce("min", g, O.SRC, x, n)[2] == np.finfo(np.float32).max).all()
    assert (O.copy_reduce("sum", g, O.SRC, x, n)[0] == 0).all()
    assert (O.copy_reduce("mean", g, O.SRC, x, n)[0] == 0).all()


def test_max_grad_to_all_ties():
    """functor.h:36-38: the max gradient goes to every tied edge."""
    src, dst, n = np.array([0, 0, 1]), np.array([2, 2, 2]), 3
    g = O.RefGraph(src, dst, n)
    x = np.array([[1.0], [1.0], [0.0]], np.float32)
    out, gx = O.copy_reduce("max", g, O.SRC, x, n, grad_out=np.ones((3, 1), np.float32))
    assert out[2, 0] == 1.0
    # node 0 feeds two tied edges, node 1 one tied edge
    np.testing.assert_array_equal(gx[:, 0], [2.0, 1.0, 0.0])


def test_golden_fixture_regression():
    """The committed golden vectors (tests/golden/make_golden.py) reproduce."""
    path = os.path.join(HERE, "golden", "kernel_g20.npz")
    z = np.load(path, allow_pickle=False)
    import make_golden  # noqa: E402
    for name, arrs in make_golden.cases():
        for k, v in arrs.items():
            np.testing.assert_allclose(v, z[name + "/" + k], rtol=1e-6, atol=1e-6, err_msg=name + "/" + k)


def test_star_graph_known_answers():
    """tests/compute/test_function.py:5-67: the reference's star graph (0 -> 1..8 ->
    9 -> 0), node features 1..10 and its literal edge features; copy_src / copy_edge /
    src_mul_edge summed into each node give the test's literal vectors."""
    src = [s for i in range(1, 9) for s in (0, i)] + [9]
    dst = [d for i in range(1, 9) for d in (i, 9)] + [0]
    g = O.RefGraph(np.array(src), np.array(dst), 10)
    h = np.arange(1, 11, dtype=np.float32).reshape(10, 1)
    eh = np.array([1., 2., 1., 3., 1., 4., 1., 5., 1., 6., 1., 7., 1., 8., 1., 9., 10.],
                  np.float32).reshape(17, 1)
    copy_ans = [10., 1., 1., 1., 1., 1., 1., 1., 1., 44.]
    out = O.copy_reduce("sum", g, O.SRC, h, 10)
    _eq(out[:, 0], copy_ans)
    out = O.copy_reduce("sum", g, O.EDGE, eh, 10)
    _eq(out[:, 0], copy_ans)
    out = O.binary_reduce("sum", "mul", g, O.SRC, O.EDGE, h, eh, 10)
    _eq(out[:, 0], [100., 1., 1., 1., 1., 1., 1., 1., 1., 284.])


SPECIAL = json.load(open(os.path.join(HERE, "golden", "special_values.json")))


@pytest.mark.parametrize("red", ["sum", "max", "min"])
def test_special_values_known_answers(red):
    """NaN / +-inf / zero-in-degree rows: the oracle follows std::max / std::min
    exactly (functor.h:33,44 -- a NaN message never replaces the accumulator)
    and the identity fill; known answers from tests/golden/make_special.py."""
    d = SPECIAL
    x = np.array(d["x"], np.float32)
    ref = O.RefGraph(np.array(d["src"]), np.array(d["dst"]), d["n"])
    for nthreads in (1, 4):
        out, gx = O.copy_reduce(red, ref, O.SRC, x, d["n"], grad_out=np.ones_like(x),
                                nthreads=nthreads)
        np.testing.assert_array_equal(out, np.array(d["cases"][red]["out"], np.float32))
        np.testing.assert_array_equal(gx, np.array(d["cases"][red]["grad_x"], np.float32))


def test_special_values_edge_softmax():
    """Masked (all -inf), NaN and +inf logits through the reference's edge_softmax
    decomposition (softmax.py:33-78): NaN rows where the reference makes NaN."""
    sm = SPECIAL["softmax"]
    ref = O.RefGraph(np.array(sm["src"]), np.array(sm["dst"]), SPECIAL["n"])
    s = np.array(sm["score"], np.float32).reshape(-1, 1)
    got = O.edge_softmax(ref, s).reshape(-1)
    np.testing.assert_allclose(got, np.array(sm["out"], np.float32), rtol=1e-6, equal_nan=True)
