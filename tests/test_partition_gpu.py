"""Device label-propagation partitioner (``DGLMIPartitionLabelProp``, the METIS
stand-in of ``dgl.distributed.partition_labelprop``): bit-exact against its numpy
restatement (``tests/lp_ref.py``), deterministic, balanced, better than the
contiguous split it starts from; partitions built from its assignment aggregate
exactly like the whole graph (two gloo ranks sharing cuda:0)."""
import numpy as np
import pytest
import torch as th

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _gidx(src, dst, n):
    from dgl.graph_index import device_block_gidx
    return device_block_gidx(n, n, th.from_numpy(src).to(DEV).int(), th.from_numpy(dst).to(DEV).int())


@pytest.mark.parametrize("k,balance", [(2, "edges"), (4, "nodes"), (8, "edges"), (5, "edges")])
def test_labelprop_matches_restatement(k, balance):
    from dgl import distributed as D
    from graphs import powerlaw
    from lp_ref import labelprop
    src, dst, n = powerlaw(3000, 30000, seed=k)
    g = _gidx(src, dst, n)
    assign, info = D.partition_labelprop(g, k, rounds=6, slack=0.05, balance=balance, seed=7)
    init = D.contiguous_parts_device(
        (g.in_csr.degrees() + 1).int() if balance == "edges" else th.ones(n, dtype=th.int32, device=DEV),
        k).cpu().numpy()
    w = np.bincount(dst, minlength=n) + 1 if balance == "edges" else None
    lab, load, cut = labelprop(n, src, dst, k, 6, 0.05, w, 7, init)
    np.testing.assert_array_equal(assign.cpu().numpy(), lab)
    assert info["loads"] == load.tolist()
    assert info["cut_edges"] == cut


def test_labelprop_deterministic_balanced_and_better():
    from dgl import distributed as D
    from graphs import powerlaw
    src, dst, n = powerlaw(200_000, 2_000_000, seed=11)
    g = _gidx(src, dst, n)
    k = 8
    a1, i1 = D.partition_labelprop(g, k, rounds=24, slack=0.05)
    a2, i2 = D.partition_labelprop(g, k, rounds=24, slack=0.05)
    assert th.equal(a1, a2) and i1 == i2
    w = np.bincount(dst, minlength=n) + 1
    cap = 1.05 * w.sum() / k
    assert max(i1["loads"]) <= cap * 1.02, (i1["loads"], cap)
    assert sum(i1["loads"]) == w.sum()
    s, d = th.from_numpy(src).to(DEV), th.from_numpy(dst).to(DEV)
    st = D.partition_stats(s, d, a1, k)
    ct = D.partition_stats(s, d, D.contiguous_parts_device(th.from_numpy(w).int().to(DEV), k), k)
    assert st["cut_edges"] == i1["cut_edges"]
    assert st["cut_edges"] < 0.9 * ct["cut_edges"], (st, ct)
    assert sum(st["halo_rows"]) < sum(ct["halo_rows"])


def test_labelprop_rejects_bad_input():
    from dgl import distributed as D
    from dgl._ffi import DGLError
    from graphs import powerlaw
    src, dst, n = powerlaw(500, 3000, seed=1)
    g = _gidx(src, dst, n)
    with pytest.raises(DGLError, match="num_parts"):
        D.partition_labelprop(g, 65)
    bad = th.full((n,), 3, dtype=th.int32, device=DEV)
    with pytest.raises(DGLError, match="outside"):
        D.partition_labelprop(g, 2, init=bad)


def _agg_worker(rank, world, src, dst, n, q, exchange="pull", empty_part=False):
    import torch.distributed as dist
    from dgl import distributed as D
    from dgl import kernel as K
    s, d = th.from_numpy(src).to(DEV).int(), th.from_numpy(dst).to(DEV).int()
    g = D.device_block_gidx(n, n, s, d)
    if empty_part:  # parts {0, world-1} only: the middle ranks own nothing
        assign, _ = D.partition_labelprop(g, 2, rounds=10)
        assign = assign * (world - 1)
    else:
        assign, _ = D.partition_labelprop(g, world, rounds=10)
    part = D.build_partition_from_assignment(s, d, assign, rank, None, world, exchange=exchange,
                                             tau=2)
    x = th.from_numpy(np.random.RandomState(0).randn(n, 32).astype(np.float32)).to(DEV)
    ref = th.empty(n, 32, device=DEV)
    K.copy_reduce("sum", g, 0, x, ref)
    mass = th.empty(n, 32, device=DEV)  # sum |terms| per row: the fp32 reorder bound's scale
    K.copy_reduce("sum", g, 0, x.abs(), mass)
    x_inner = x[part.inner_global].contiguous()
    if exchange == "hybrid":
        out = D.aggregate_hybrid(x_inner, part)
        out2 = D.aggregate_hybrid(x_inner, part)
        full_exact = bool(th.equal(out, out2))  # deterministic
        n_push = part.n_pin
    else:
        out = D.aggregate_with_halo(x_inner, part)
        full = D.halo_exchange(x_inner, part)  # autograd path: [owned | halo] rows
        full_exact = bool(th.equal(full, th.cat([x_inner, x[part.halo_global]])))
        n_push = 0
    bound = 1e-5 + 2e-6 * mass[part.inner_global]
    rel = (out - ref[part.inner_global]).abs() / bound
    res = {"err": float(rel.max()) if rel.numel() else 0.0,
           "full_exact": full_exact, "inner": part.inner, "n_halo": part.n_halo,
           "n_push": n_push}
    objs = [None] * world
    dist.all_gather_object(objs, res)
    if rank == 0:
        inner = np.concatenate([o["inner"] for o in objs])
        assert np.array_equal(np.sort(inner), np.arange(n))
        assert all(o["full_exact"] for o in objs)
        assert max(o["err"] for o in objs) <= 1.0  # within the mass-scaled bound
        if exchange == "hybrid":
            assert sum(o["n_push"] for o in objs) > 0  # the push side was exercised
        q.put("ok")


@pytest.mark.parametrize("exchange,world,empty", [("pull", 2, False), ("hybrid", 2, False),
                                                  ("hybrid", 3, False), ("hybrid", 3, True),
                                                  ("pull", 3, True)])
def test_labelprop_partitioned_aggregation_matches_single_gpu(exchange, world, empty):
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(5000, 60000, seed=5)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_agg_worker, world, (src, dst, n, q, exchange, empty))
    assert q.get(timeout=5) == "ok"


def test_metis_partition_on_gpu_uses_label_propagation():
    """dgl.transform.metis_partition with a GPU present partitions with the device
    label propagation (node-balanced like METIS); the reference's structural checks
    (tests/compute/test_transform.py:245-274) hold, and parts stay within 3 %."""
    import dgl
    from dgl import distributed as D
    rng = np.random.default_rng(0)
    n = 1000
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(rng.integers(0, n, n * 10), rng.integers(0, n, n * 10))
    for hops in (0, 1):
        subgs = dgl.transform.metis_partition(g, 4, hops)
        inner_total = 0
        for pid, sub in subgs.items():
            inner = sub.ndata["inner_node"].numpy()
            inner_total += int(inner.sum())
            assert (sub.ndata["part_id"].numpy()[inner == 1] == pid).all()
            if hops == 0:
                assert (inner == 1).all() and (sub.edata["inner_edge"].numpy() == 1).all()
            assert int(inner.sum()) <= 1.03 * n / 4 + 1
        assert inner_total == n
    s, d = (t.numpy() for t in g.edges())
    a = D.partition_assignment(n, s, d, 4, "labelprop")
    assert a.min() >= 0 and a.max() < 4
