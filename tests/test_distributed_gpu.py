"""Partition-parallel 2-layer GCN (halo exchange + gradient all-reduce) equals the
single-GPU model.  Two ranks share cuda:0 (gloo collectives) -- the 8-GPU RCCL
run is the driver's; this checks the math of the distributed path."""
import numpy as np
import pytest
import torch as th

pytestmark = pytest.mark.gpu


def _model(fin, hid, fout):
    from dgl.nn.pytorch import GraphConv
    th.manual_seed(0)
    return GraphConv(fin, hid, activation=th.relu), GraphConv(hid, fout)


def _worker(rank, world, src, dst, n, q, planner):
    import dgl
    from dgl import distributed as D
    dev = "cuda:0"
    c1, c2 = _model(16, 32, 8)
    d1, d2 = D.DistGraphConv(16, 32, activation=th.relu), D.DistGraphConv(32, 8)
    d1.conv.load_state_dict(c1.state_dict())
    d2.conv.load_state_dict(c2.state_dict())
    d1, d2 = d1.to(dev), d2.to(dev)
    if planner == "host_ldg":
        assign = D.partition_assignment(n, src, dst, world, "ldg")
        part = D.build_partitions(src, dst, n, assign, num_parts=world)[rank]
    elif planner == "device_lp_hybrid":  # label propagation + pull / push-partial exchange
        s_d, d_d = th.from_numpy(src).to(dev).int(), th.from_numpy(dst).to(dev).int()
        assign, _ = D.partition_labelprop(D.device_block_gidx(n, n, s_d, d_d), world, rounds=8)
        part = D.build_partition_from_assignment(s_d, d_d, assign, rank, None, world,
                                                 exchange="hybrid", tau=2)
    else:  # contiguous id ranges, halo plan built on the device
        bounds = [n * p // world for p in range(world + 1)]
        lo, hi = bounds[rank], bounds[rank + 1]
        sel = (dst >= lo) & (dst < hi)
        part = D.build_device_partition(th.from_numpy(src[sel]).to(dev).int(),
                                        th.from_numpy(dst[sel] - lo).to(dev).int(), bounds, rank)
    x = th.from_numpy(np.random.RandomState(0).randn(n, 16).astype(np.float32))
    inner = th.from_numpy(part.inner)
    odeg = th.from_numpy(np.bincount(src, minlength=n))[inner].to(dev)
    ideg = th.from_numpy(np.bincount(dst, minlength=n))[inner].to(dev)
    h = d1(part, x[inner].to(dev), odeg, ideg)
    out = d2(part, h, odeg, ideg)
    out.pow(2).sum().backward()
    params = list(d1.parameters()) + list(d2.parameters())
    D.allreduce_gradients(params, average=False)
    res = {"rank": rank, "inner": part.inner, "out": out.detach().cpu().numpy(),
           "grads": [p.grad.detach().cpu().numpy() for p in params]}
    import torch.distributed as dist
    objs = [None] * world
    dist.all_gather_object(objs, res)
    if rank == 0:
        # single-GPU reference on the whole graph
        g = dgl.DGLGraph()
        g.add_nodes(n)
        g.add_edges(src, dst)
        c1d, c2d = c1.to(dev), c2.to(dev)
        ref = c2d(g, c1d(g, x.to(dev)))
        ref.pow(2).sum().backward()
        rg = [p.grad.cpu().numpy() for p in list(c1d.parameters()) + list(c2d.parameters())]
        full = np.zeros((n, 8), np.float32)
        for o in objs:
            full[o["inner"]] = o["out"]
        np.testing.assert_allclose(full, ref.detach().cpu().numpy(), rtol=1e-4, atol=1e-4)
        for a, b in zip(objs[0]["grads"], rg):
            np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-3)
        q.put("ok")


@pytest.mark.parametrize("planner", ["host_ldg", "device_contiguous", "device_lp_hybrid"])
def test_dist_gcn_matches_single_gpu(planner):
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 40000, seed=3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_worker, 2, (src, dst, n, q, planner))
    assert q.get(timeout=5) == "ok"


def _overlap_worker(rank, world, src, dst, n, q):
    import dgl
    from dgl import distributed as D
    dev = "cuda:0"
    bounds = [n * p // world for p in range(world + 1)]
    lo, hi = bounds[rank], bounds[rank + 1]
    sel = (dst >= lo) & (dst < hi)
    part = D.build_device_partition(th.from_numpy(src[sel]).to(dev).int(),
                                    th.from_numpy(dst[sel] - lo).to(dev).int(), bounds, rank)
    x = th.from_numpy(np.random.RandomState(1).randn(n, 16).astype(np.float32)).to(dev)
    out = D.aggregate_with_halo(x[lo:hi].contiguous(), part)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    gi = g._graph.get_immutable_gidx(dev)
    ref = dgl.backend.copy_reduce("sum", gi, 0, x, n)[lo:hi]
    # fp32 reorder bound: the two sums add the same terms in different orders
    mass = dgl.backend.copy_reduce("sum", gi, 0, x.abs(), n)[lo:hi]
    ok = bool(((out - ref).abs() <= 1e-5 + 2e-6 * mass).all())
    import torch.distributed as dist
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    if rank == 0:
        q.put("ok" if all(flags) else "mismatch")


def test_aggregate_with_halo_overlapped():
    """Owned-source half + halo half (accumulated by the kernel's addend epilogue)
    == the full aggregation of the owned rows, 2 ranks on one GPU."""
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 40000, seed=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_overlap_worker, 2, (src, dst, n, q))
    assert q.get(timeout=5) == "ok"


def _gat_rgcn_worker(rank, world, src, dst, et, n, q, planner, fin=16, fout=8):
    import dgl
    from dgl import distributed as D
    from dgl.nn.pytorch import GATConv, RelGraphConv
    dev = "cuda:0"
    R = 3
    th.manual_seed(0)
    gat = GATConv(fin, 8, 4).to(dev)
    rel = RelGraphConv(fin, fout, R, "basis", num_bases=2, self_loop=True).to(dev)
    dg = D.DistGATConv(fin, 8, 4).to(dev)
    dr = D.DistRelGraphConv(fin, fout, R, "basis", num_bases=2, self_loop=True).to(dev)
    dg.conv.load_state_dict(gat.state_dict())
    dr.conv.load_state_dict(rel.state_dict())
    et_t = th.from_numpy(et).to(dev)
    norm = th.from_numpy(1.0 / np.maximum(np.bincount(dst, minlength=n), 1)[dst]).float().to(dev)
    norm = norm.view(-1, 1)
    if planner == "host_ldg":
        assign = D.partition_assignment(n, src, dst, world, "ldg")
        part = D.build_partitions(src, dst, n, assign, num_parts=world)[rank]
        et_l, norm_l = part.local_edge_data(et_t), part.local_edge_data(norm)
    elif planner == "device_lp":  # label propagation, renumbered partition, pull exchange
        s_d, d_d = th.from_numpy(src).to(dev).int(), th.from_numpy(dst).to(dev).int()
        assign, _ = D.partition_labelprop(D.device_block_gidx(n, n, s_d, d_d), world, rounds=8)
        part = D.build_partition_from_assignment(s_d, d_d, assign, rank, None, world)
        keep = assign[d_d.long()] == rank  # local edge order: the global order, kept edges
        et_l, norm_l = et_t[keep], norm[keep]
    else:
        bounds = [n * p // world for p in range(world + 1)]
        lo, hi = bounds[rank], bounds[rank + 1]
        sel = (dst >= lo) & (dst < hi)
        part = D.build_device_partition(th.from_numpy(src[sel]).to(dev).int(),
                                        th.from_numpy(dst[sel] - lo).to(dev).int(), bounds, rank)
        idx = th.from_numpy(np.nonzero(sel)[0]).to(dev)
        et_l, norm_l = et_t[idx], norm[idx]
    x = th.from_numpy(np.random.RandomState(2).randn(n, fin).astype(np.float32)).to(dev)
    inner = th.from_numpy(part.inner).to(dev)
    xi = x[inner]
    og = dg(part, xi)
    orl = dr(part, xi, et_l, norm_l)
    fused = part.local_graph(dev)._graph.__dict__.get("_rgcn_fused") is not None
    assert fused == (fin == 64 and fout == 64)  # the fused R-GCN route on the local block
    (og.pow(2).sum() + orl.pow(2).sum()).backward()
    params = list(dg.parameters()) + list(dr.parameters())
    D.allreduce_gradients(params, average=False)
    res = {"inner": part.inner, "g": og.detach().cpu().numpy(), "r": orl.detach().cpu().numpy(),
           "grads": [p.grad.detach().cpu().numpy() for p in params]}
    import torch.distributed as dist
    objs = [None] * world
    dist.all_gather_object(objs, res)
    if rank == 0:
        g = dgl.DGLGraph()
        g.add_nodes(n)
        g.add_edges(src, dst)
        rg = gat(g, x)
        rr = rel(g, x, et_t, norm)
        (rg.pow(2).sum() + rr.pow(2).sum()).backward()
        ref_grads = [p.grad.cpu().numpy() for p in list(gat.parameters()) + list(rel.parameters())]
        full_g = np.zeros(tuple(rg.shape), np.float32)
        full_r = np.zeros(tuple(rr.shape), np.float32)
        for o in objs:
            full_g[o["inner"]] = o["g"]
            full_r[o["inner"]] = o["r"]
        np.testing.assert_allclose(full_g, rg.detach().cpu().numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(full_r, rr.detach().cpu().numpy(), rtol=1e-4, atol=1e-4)
        for a, b in zip(objs[0]["grads"], ref_grads):
            # long fp32 sums (tens of thousands of terms) in other orders: scaled bound
            assert np.abs(a - b).max() <= 1e-3 + 1e-4 * np.abs(b).max()
        q.put("ok")


@pytest.mark.parametrize("planner", ["host_ldg", "device_contiguous"])
def test_dist_rgcn_fused_route_matches_single_gpu(planner):
    """DistRelGraphConv 64 -> 64 runs the fused R-GCN kernels on each rank's local
    block (owned + halo rows): outputs and all-reduced gradients equal the
    whole-graph module's, 2 ranks on one GPU."""
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 40000, seed=7)
    et = np.random.default_rng(7).integers(0, 3, len(src))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_gat_rgcn_worker, 2, (src, dst, et, n, q, planner, 64, 64))
    assert q.get(timeout=5) == "ok"


@pytest.mark.parametrize("planner", ["host_ldg", "device_contiguous", "device_lp"])
def test_dist_gat_and_rgcn_match_single_gpu(planner):
    """DistGATConv (fused GAT on the local block, ft/el halo rows exchanged) and
    DistRelGraphConv (x halo rows exchanged, typed gather on the local block):
    outputs and all-reduced weight gradients equal the whole-graph modules."""
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 40000, seed=5)
    et = np.random.default_rng(5).integers(0, 3, len(src))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_gat_rgcn_worker, 2, (src, dst, et, n, q, planner))
    assert q.get(timeout=5) == "ok"


def _rccl_world1_worker(rank, world, src, dst, et, n, q):
    """Every collective of the distributed path on RCCL (backend "nccl", device
    tensors, async all-to-all-v on the collective stream) at world size 1: the GCN
    with all three planners, the overlapped aggregation and DistGAT / DistRelGraphConv."""
    import torch.distributed as dist
    assert dist.get_backend() == "nccl"
    for planner in ("host_ldg", "device_contiguous", "device_lp_hybrid"):
        _worker(rank, world, src, dst, n, q, planner)
    _overlap_worker(rank, world, src, dst, n, q)
    for planner in ("host_ldg", "device_contiguous", "device_lp"):
        _gat_rgcn_worker(rank, world, src, dst, et, n, q, planner)


def test_rccl_world1_collectives():
    """The N>1 runs use RCCL, which refuses two ranks on one GPU; a world of one
    rank still drives every RCCL call of the path (halo all-to-all-v with zero
    splits, gradient all-reduce, all_gather_object) on the device."""
    import torch.multiprocessing as mp
    from dist_util import run_world
    from graphs import powerlaw
    src, dst, n = powerlaw(3000, 40000, seed=6)
    et = np.random.default_rng(6).integers(0, 3, len(src))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    run_world(_rccl_world1_worker, 1, (src, dst, et, n, q), backend="nccl")
    got = [q.get(timeout=5) for _ in range(7)]
    assert got == ["ok"] * 7, got
