"""Partition + halo exchange + gradient all-reduce with gloo, world_size 2 (CPU)."""
import numpy as np
import pytest
import torch as th

from dgl import distributed as D
from graphs import powerlaw
from dist_util import run_world


@pytest.mark.parametrize("method", ["contiguous", "ldg"])
@pytest.mark.parametrize("k", [2, 3, 4])
def test_partitions_cover_graph(method, k):
    src, dst, n = powerlaw(3000, 30000, seed=4)
    assign = D.partition_assignment(n, src, dst, k, method)
    assert assign.min() >= 0 and assign.max() < k
    parts = D.build_partitions(src, dst, n, assign, num_parts=k)
    seen = np.concatenate([p.parent_eid for p in parts])
    assert np.array_equal(np.sort(seen), np.arange(len(src)))  # every edge exactly once
    for p in parts:
        full = np.concatenate([p.inner, p.halo])
        np.testing.assert_array_equal(full[p.local_src], src[p.parent_eid])
        np.testing.assert_array_equal(p.inner[p.local_dst], dst[p.parent_eid])
        assert (assign[p.inner] == p.part_id).all() and (assign[p.halo] != p.part_id).all()
        # send plan of q towards p == p's halo rows owned by q, in p's order
        for q in parts:
            if q.part_id == p.part_id:
                continue
            off = int(q.send_counts[:p.part_id].sum())
            rows = q.inner[q.send_idx[off:off + q.send_counts[p.part_id]]]
            np.testing.assert_array_equal(rows, p.halo[p.halo_owner == q.part_id])
    if method == "ldg":
        sizes = np.bincount(assign, minlength=k)
        assert sizes.max() <= np.ceil(n / k) * 1.05 + 1


def test_ldg_cuts_fewer_edges_than_random():
    """A graph with 4 planted communities (ids shuffled): LDG must cut far fewer
    edges than a random assignment."""
    rng = np.random.default_rng(0)
    n, m = 400, 8000
    block = rng.permutation(np.repeat(np.arange(4), n // 4))
    members = [np.nonzero(block == b)[0] for b in range(4)]
    u = rng.integers(0, n, m)
    intra = rng.random(m) < 0.9
    v = np.where(intra, np.array([rng.choice(members[block[x]]) for x in u]), rng.integers(0, n, m))
    a_ldg = D.partition_assignment(n, u, v, 4, "ldg")
    a_rand = rng.integers(0, 4, n)
    cut = lambda a: int((a[u] != a[v]).sum())
    assert cut(a_ldg) < 0.6 * cut(a_rand)


def _halo_worker(rank, world, src, dst, n, k):
    import torch.distributed as dist
    assign = D.partition_assignment(n, src, dst, k, "ldg")
    part = D.build_partitions(src, dst, n, assign, num_parts=k)[rank]
    g = th.Generator().manual_seed(0)
    xg = th.randn(n, 5, generator=g)
    wg = th.randn(n, 5, generator=g)
    x_inner = xg[th.from_numpy(part.inner)].clone().requires_grad_()
    full = D.halo_exchange(x_inner, part)
    ids = th.from_numpy(np.concatenate([part.inner, part.halo]))
    assert th.equal(full.detach(), xg[ids])
    # loss = sum over every (local use) of w * x ; the gradient of an owned row must
    # collect the uses on every rank that holds it as halo
    (full * wg[ids]).sum().backward()
    uses = th.zeros(n)
    for p in D.build_partitions(src, dst, n, assign, num_parts=k):
        uses.index_add_(0, th.from_numpy(np.concatenate([p.inner, p.halo])), th.ones(p.n_inner + p.n_halo))
    expect = wg[th.from_numpy(part.inner)] * uses[th.from_numpy(part.inner)][:, None]
    assert th.allclose(x_inner.grad, expect, atol=1e-6)
    # flattened gradient all-reduce
    p1 = th.nn.Parameter(th.zeros(3, 2))
    p2 = th.nn.Parameter(th.zeros(4))
    p1.grad = th.full((3, 2), float(rank + 1))
    p2.grad = th.full((4,), float(10 * (rank + 1)))
    D.allreduce_gradients([p1, p2])
    assert th.allclose(p1.grad, th.full((3, 2), sum(r + 1 for r in range(world)) / world))
    assert th.allclose(p2.grad, th.full((4,), sum(10 * (r + 1) for r in range(world)) / world))
    dist.barrier()


def test_halo_exchange_gloo_world2():
    src, dst, n = powerlaw(500, 4000, seed=1)
    run_world(_halo_worker, 2, (src, dst, n, 2))


def _device_plan_worker(rank, world, src, dst, n):
    bounds = [n * p // world for p in range(world + 1)]
    assign = np.searchsorted(np.asarray(bounds[1:]), np.arange(n), side="right")
    ref = D.build_partitions(src, dst, n, assign, num_parts=world)[rank]
    lo, hi = bounds[rank], bounds[rank + 1]
    sel = (dst >= lo) & (dst < hi)
    part = D.build_device_partition(th.from_numpy(src[sel]).int(), th.from_numpy(dst[sel] - lo).int(),
                                    bounds, rank)
    # same halo set / order, same exchange plan and local numbering as the host planner
    assert part.n_inner == ref.n_inner and part.n_halo == ref.n_halo
    assert np.array_equal(part.halo.numpy(), ref.halo)
    assert np.array_equal(part.send_counts, ref.send_counts)
    assert np.array_equal(part.recv_counts, ref.recv_counts)
    assert np.array_equal(part.send_idx.numpy(), ref.send_idx)
    assert np.array_equal(part.local_src.numpy(), ref.local_src)
    assert np.array_equal(part.local_dst.numpy(), ref.local_dst)
    # in-place exchange fills the halo rows with the owners' features
    xg = th.randn(n, 3, generator=th.Generator().manual_seed(1))
    full = th.empty(part.n_inner + part.n_halo, 3)
    full[:part.n_inner] = xg[lo:hi]
    D.halo_exchange_into(full, part)
    assert th.equal(full[part.n_inner:], xg[part.halo])


@pytest.mark.parametrize("world", [2, 3])
def test_device_partition_plan_matches_host(world):
    src, dst, n = powerlaw(700, 6000, seed=3)
    run_world(_device_plan_worker, world, (np.asarray(src), np.asarray(dst), n))


def _ldg_agg_worker(rank, world, src, dst, n):
    """LDG partition -> halo exchange -> local aggregation over the partition's
    block equals the whole-graph aggregation (sum over in-edges) on the owned rows.
    The local sum is torch's index_add (CPU stand-in for the HIP copy_u_sum the
    GPU tests run)."""
    import torch.distributed as dist
    assign = D.partition_assignment(n, src, dst, world, "ldg")
    part = D.build_partitions(src, dst, n, assign, num_parts=world)[rank]
    xg = th.randn(n, 4, generator=th.Generator().manual_seed(2), dtype=th.float64)
    full = D.halo_exchange(xg[th.from_numpy(part.inner)].clone(), part)
    local = th.zeros(part.n_inner, 4, dtype=th.float64).index_add_(
        0, th.from_numpy(part.local_dst), full[th.from_numpy(part.local_src)])
    ref = th.zeros(n, 4, dtype=th.float64).index_add_(0, th.from_numpy(dst), xg[th.from_numpy(src)])
    assert th.allclose(local, ref[th.from_numpy(part.inner)], atol=1e-9)
    # LDG cuts fewer edges than the contiguous split of the same (permuted-id) graph
    ct = D.partition_assignment(n, src, dst, world, "contiguous")
    assert (assign[src] != assign[dst]).sum() < (ct[src] != ct[dst]).sum()
    dist.barrier()


def test_ldg_partitioned_aggregation_gloo_world2():
    rng = np.random.default_rng(7)
    n = 2000
    # communities hidden behind a random id permutation
    block = rng.permutation(np.repeat(np.arange(2), n // 2))
    u = rng.integers(0, n, 20000)
    same = rng.random(20000) < 0.8
    members = [np.nonzero(block == b)[0] for b in range(2)]
    v = np.where(same, np.array([rng.choice(members[block[x]]) for x in u]), rng.integers(0, n, 20000))
    run_world(_ldg_agg_worker, 2, (u.astype(np.int64), v.astype(np.int64), n))


def _hybrid_plan_worker(rank, world, src, dst, n, tau, bounds=None):
    """The hybrid (pull + push-partial) plan, executed with torch index_add on the
    CPU (stand-in for the HIP SpMMs of aggregate_hybrid): every in-edge of an owned
    destination is summed exactly once over all ranks, so the result equals the
    whole-graph sum; x = ones counts the in-degrees exactly."""
    import torch.distributed as dist
    if bounds is None:
        bounds = [n * p // world for p in range(world + 1)]
    lo, hi = bounds[rank], bounds[rank + 1]
    sel = (dst >= lo) & (dst < hi)
    pl = D.plan_hybrid(th.from_numpy(src[sel]), th.from_numpy(dst[sel] - lo), bounds, rank,
                       None, tau)
    xg = th.randn(n, 3, generator=th.Generator().manual_seed(4), dtype=th.float64)
    results = []
    for x in (xg, th.ones(n, 3, dtype=th.float64)):
        xi = x[lo:hi]
        send = xi[pl["send_idx"]]
        recv_pull = th.empty(pl["n_halo"], 3, dtype=th.float64)
        D._a2av(recv_pull, send, pl["recv_counts"].tolist(), pl["send_counts"].tolist(), None)
        pout = th.zeros(pl["n_pout"], 3, dtype=th.float64).index_add_(0, pl["push_row"],
                                                                       xi[pl["push_src"]])
        recv_part = th.empty(pl["n_pin"], 3, dtype=th.float64)
        D._a2av(recv_part, pout, pl["pin_counts"].tolist(), pl["pout_counts"].tolist(), None)
        recv = th.cat([recv_pull, recv_part])
        out = th.zeros(hi - lo, 3, dtype=th.float64).index_add_(0, pl["own_dst"], xi[pl["own_src"]])
        out.index_add_(0, pl["recv_dst"], recv[pl["recv_col"]])
        results.append(out)
    ref = th.zeros(n, 3, dtype=th.float64).index_add_(0, th.from_numpy(dst), xg[th.from_numpy(src)])
    assert th.allclose(results[0], ref[lo:hi], atol=1e-9)
    indeg = th.from_numpy(np.bincount(dst, minlength=n)[lo:hi]).double()
    assert th.equal(results[1][:, 0], indeg)
    flags = [None] * world
    dist.all_gather_object(flags, (pl["n_pin"], pl["n_halo"]))
    assert sum(f[0] for f in flags) > 0  # partial rows were exercised


@pytest.mark.parametrize("world,tau", [(2, 2), (3, 3), (2, 8)])
def test_hybrid_plan_gloo(world, tau):
    src, dst, n = powerlaw(3000, 40000, seed=6)
    run_world(_hybrid_plan_worker, world, (src, dst, n, tau))


def test_hybrid_plan_gloo_empty_part():
    """A rank that owns no nodes (bounds [0, n/2, n/2, n]) sends and receives
    nothing, and the two others still sum every in-edge exactly once."""
    src, dst, n = powerlaw(2000, 30000, seed=9)
    run_world(_hybrid_plan_worker, 3, (src, dst, n, 4, [0, n // 2, n // 2, n]))
