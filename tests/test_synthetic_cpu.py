"""Host-side seeded draws: the Chung-Lu edge lists every rank of a multi-GPU bench
builds on its own (dgl.data.synthetic.chung_lu_edges: the same draw on every call, in
range, skewed like the power law it samples) and the fused GAT's attention-dropout
mask (dgl.kernel.gat_dropout_keep)."""
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


def test_gat_dropout_keep_mask_statistics():
    """The fused GAT's attention-dropout mask (host mirror of the kernel's hash): the
    kept share is 1 - p, heads and seeds give independent draws."""
    import numpy as np
    from dgl.kernel import gat_dropout_keep
    eids = np.arange(250_000)
    for p in (0.1, 0.5, 0.6):
        k = gat_dropout_keep(12345, eids, 8, p)
        assert k.shape == (250_000, 8)
        assert abs(k.mean() - (1 - p)) < 0.005
        # no two heads of one edge are correlated (heads 2j / 2j + 1 share one hash:
        # its low and high halves), nor neighbouring edge ids
        for i in range(8):
            assert abs(k[:, i].mean() - (1 - p)) < 0.006
            for j in range(i + 1, 8):
                assert abs((k[:, i] & k[:, j]).mean() - (1 - p) ** 2) < 0.006, (i, j)
        assert abs((k[1:, 0] & k[:-1, 0]).mean() - (1 - p) ** 2) < 0.006
    a, b = gat_dropout_keep(1, eids, 4, 0.5), gat_dropout_keep(2, eids, 4, 0.5)
    assert abs((a == b).mean() - 0.5) < 0.01
    assert gat_dropout_keep(7, eids[:10], 4, 0.0).all()
