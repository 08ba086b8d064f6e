"""The seeded Chung-Lu edge lists every rank of a multi-GPU bench builds on its own
(dgl.data.synthetic.chung_lu_edges): the same draw on every call, in range, and
skewed like the power law it samples."""
import torch as th

from dgl.data.synthetic import chung_lu_edges


def test_chung_lu_edges_repeatable_and_skewed():
    n, m = 20_000, 400_000
    a = chung_lu_edges(n, m, 0.5, 8, "cpu")
    b = chung_lu_edges(n, m, 0.5, 8, "cpu")
    c = chung_lu_edges(n, m, 0.5, 9, "cpu")
    for x, y in zip(a, b):
        assert x.dtype == th.int32 and th.equal(x, y)
    assert not th.equal(a[0], c[0])
    for x in a:
        assert int(x.min()) >= 0 and int(x.max()) < n
    # expected degree of node i is m * w_i / sum(w): the heaviest node gets
    # ~ m / sum_{k<=n} k^-0.5 ~ m / (2 sqrt(n)) = 1414 ends; a uniform draw gives ~20
    deg = th.bincount(a[1].long(), minlength=n)
    assert 1000 < int(deg.max()) < 2000
    # the two ends are independent draws
    assert not th.equal(a[0], a[1])
