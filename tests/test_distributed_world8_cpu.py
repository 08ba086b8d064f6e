"""The 8-rank topology of config C4 (one node, 8 GPUs) rehearsed with gloo on the CPU,
world sizes 4 and 8: every collective, buffer and index of the partitioned aggregation
runs as on the node; only the three per-rank copy_u_sum blocks and the block CSRs are
torch stand-ins (index_add over the block's edge list -- the GPU tests run the HIP
kernels at world 2 / 3 on one card).  Checked against the single-process whole-graph
result on every rank:

* the host and the device halo planners agree at world 4 / 8 (test_distributed_cpu.py);
* ``aggregate_with_halo`` (pull exchange, owned block overlapping the all-to-all-v),
  ``aggregate_hybrid`` (pull + push-partial, tau = 2 and 8) and the differentiable
  ``hybrid_aggregate`` (GraphConv's norm / bias epilogue; its backward's reverse
  exchanges) -- including worlds where some ranks own no nodes at all;
* ``build_partition_from_assignment`` for an arbitrary (non-contiguous) assignment,
  both exchanges, results mapped back through ``inner_global``;
* ``allreduce_gradients`` (one flattened all-reduce) at world 8.

The reference's halo semantics: ``src/graph/graph_op.cc:403-509`` (num_hops = 1: a part
owns its nodes and all their in-edges); its multi-GPU pattern
``examples/pytorch/graphsage/train_sampling_multi_gpu.py:190-270``."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch as th

from dgl import distributed as D
from graphs import powerlaw
from dist_util import run_world


# --------------------------------------------------------------------------- #
# CPU stand-ins for the per-rank kernels (installed inside each worker process)
# --------------------------------------------------------------------------- #
class CpuBlock:
    """A (num_src -> num_dst) block as an edge list: what device_block_gidx builds."""

    def __init__(self, num_src, num_dst, src, dst, bits=None):
        self.num_src, self.num_dst = int(num_src), int(num_dst)
        self.src, self.dst = src.long(), dst.long()
        assert (self.src.numel() == 0 or int(self.src.max()) < self.num_src)
        assert (self.dst.numel() == 0 or int(self.dst.max()) < self.num_dst)
        self.in_csr = SimpleNamespace(indices=src.to(th.int32), rows=dst.to(th.int32))

    def number_of_edges(self):
        return int(self.src.numel())


def _copy_reduce(reducer, graph, target, in_data, out_data, in_map=None, out_map=None,
                 epilogue=None):
    assert reducer == "sum" and target == 0 and in_map is None and out_map is None
    assert in_data.shape[0] == graph.num_src and out_data.shape[0] == graph.num_dst
    out = th.zeros(out_data.shape, dtype=in_data.dtype).index_add_(0, graph.dst,
                                                                   in_data[graph.src])
    if epilogue is not None:
        row_mul, row_div, bias, addend = (tuple(epilogue) + (None,) * 4)[:4]
        if row_mul is not None:
            out = out * row_mul.reshape(-1, *([1] * (out.dim() - 1)))
        if row_div is not None:
            out = out / row_div.reshape(-1, *([1] * (out.dim() - 1)))
        if bias is not None:
            out = out + bias
        if addend is not None:
            out = out + addend
    out_data.copy_(out)
    return out_data


def _backward_copy_reduce(reducer, graph, target, in_data, out_data, grad_out, grad_in,
                          in_map=None, out_map=None):
    assert reducer == "sum" and target == 0
    grad_in.copy_(th.zeros(grad_in.shape, dtype=grad_out.dtype).index_add_(
        0, graph.src, grad_out[graph.dst]))
    return grad_in


def _install_stand_ins():
    from dgl import kernel as K
    K.copy_reduce = _copy_reduce
    K.backward_copy_reduce = _backward_copy_reduce
    D.device_block_gidx = CpuBlock


def _bounds(n, world, empty=()):
    """world + 1 node-id bounds; the parts listed in ``empty`` own no nodes."""
    live = [p for p in range(world) if p not in empty]
    cuts = [n * i // len(live) for i in range(len(live) + 1)]
    b, j = [0], 0
    for p in range(world):
        if p not in empty:
            j += 1
        b.append(cuts[j])
    return b


def _whole(src, dst, n, x):
    return th.zeros((n,) + tuple(x.shape[1:]), dtype=x.dtype).index_add_(
        0, th.from_numpy(dst), x[th.from_numpy(src)])


# --------------------------------------------------------------------------- #
# forward: pull and hybrid exchanges
# --------------------------------------------------------------------------- #
def _aggregate_worker(rank, world, src, dst, n, bounds, tau):
    import torch.distributed as dist
    _install_stand_ins()
    lo, hi = bounds[rank], bounds[rank + 1]
    sel = (dst >= lo) & (dst < hi)
    s_loc = th.from_numpy(src[sel])
    d_loc = th.from_numpy(dst[sel] - lo)
    xg = th.randn(n, 6, generator=th.Generator().manual_seed(5), dtype=th.float64)
    ref = _whole(src, dst, n, xg)[lo:hi]
    xi = xg[lo:hi].contiguous()
    # pull: the halo subgraph planned on the "device", owned block overlapping the a2av
    part = D.build_device_partition(s_loc.int(), d_loc.int(), bounds, rank)
    assert part.n_inner == hi - lo
    out = D.aggregate_with_halo(xi, part)
    assert out.shape == (hi - lo, 6) and th.allclose(out, ref, atol=1e-9)
    # halo rows in place (the with-exchange line's step)
    full = th.empty(part.n_inner + part.n_halo, 6, dtype=th.float64)
    full[:part.n_inner] = xi
    D.halo_exchange_into(full, part)
    assert th.equal(full[part.n_inner:], xg[part.halo])
    # hybrid: pull + push-partial, every in-edge summed once over the ranks
    hp = D.build_hybrid_partition(s_loc, d_loc, bounds, rank, tau=tau)
    bufs = D.hybrid_buffers(xi, hp)
    out_h = D.aggregate_hybrid(xi, hp, bufs=bufs)
    assert th.allclose(out_h, ref, atol=1e-9)
    out_h2 = D.aggregate_hybrid(xi, hp, bufs=bufs)  # buffers reused: same result
    assert th.equal(out_h, out_h2)
    stats = [None] * world
    dist.all_gather_object(stats, (hp.n_pin, hp.n_pout, hp.n_halo, part.n_halo, hi - lo))
    # every partial row sent is received once; pushing never moves more rows than pulling
    assert sum(s[0] for s in stats) == sum(s[1] for s in stats)
    assert sum(s[0] + s[2] for s in stats) <= sum(s[3] for s in stats)
    if tau == 2 and all(s[4] > 0 for s in stats):
        assert sum(s[0] for s in stats) > 0  # the push side was exercised
    dist.barrier()


@pytest.mark.parametrize("world,tau,empty", [(4, 2, ()), (4, 8, (2,)), (8, 2, ()), (8, 8, ()),
                                             (8, 2, (1, 4)), (8, 8, (0, 7))])
def test_aggregate_pull_and_hybrid(world, tau, empty):
    src, dst, n = powerlaw(4000, 60000, seed=10 + world)
    run_world(_aggregate_worker, world, (src, dst, n, _bounds(n, world, empty), tau))


# --------------------------------------------------------------------------- #
# backward: the differentiable hybrid aggregation + gradient all-reduce
# --------------------------------------------------------------------------- #
def _hybrid_grad_worker(rank, world, src, dst, n, bounds, tau):
    import torch.distributed as dist
    _install_stand_ins()
    lo, hi = bounds[rank], bounds[rank + 1]
    sel = (dst >= lo) & (dst < hi)
    hp = D.build_hybrid_partition(th.from_numpy(src[sel]), th.from_numpy(dst[sel] - lo), bounds,
                                  rank, tau=tau)
    gen = th.Generator().manual_seed(8)
    xg = th.randn(n, 5, generator=gen, dtype=th.float64)
    wg = th.randn(n, 5, generator=gen, dtype=th.float64)          # d loss / d out
    norm = th.rand(n, generator=gen, dtype=th.float64) + 0.5      # GraphConv's row_mul
    bias = th.randn(5, generator=gen, dtype=th.float64)
    # whole-graph reference: out = (A x) * norm + bias, loss = sum(out * w)
    ref = _whole(src, dst, n, xg) * norm[:, None] + bias
    gx_ref = th.zeros(n, 5, dtype=th.float64).index_add_(
        0, th.from_numpy(src), (wg * norm[:, None])[th.from_numpy(dst)])
    xi = xg[lo:hi].clone().requires_grad_()
    b = bias.clone().requires_grad_()
    out = D.hybrid_aggregate(xi, hp, row_mul=norm[lo:hi].contiguous(), bias=b)
    assert th.allclose(out.detach(), ref[lo:hi], atol=1e-9)
    (out * wg[lo:hi]).sum().backward()
    # every owned row's gradient collects its uses on every rank (pulled and pushed)
    assert th.allclose(xi.grad, gx_ref[lo:hi], atol=1e-9)
    # the bias gradient all-reduced (summed) over the ranks equals the whole graph's
    D.allreduce_gradients([SimpleNamespace(grad=b.grad)], average=False)
    assert th.allclose(b.grad, wg.sum(0), atol=1e-9)
    dist.barrier()


@pytest.mark.parametrize("world,tau,empty", [(4, 2, ()), (8, 4, ()), (8, 2, (3,))])
def test_hybrid_aggregate_gradients(world, tau, empty):
    src, dst, n = powerlaw(3000, 50000, seed=20 + world)
    run_world(_hybrid_grad_worker, world, (src, dst, n, _bounds(n, world, empty), tau))


# --------------------------------------------------------------------------- #
# any assignment: renumbered parts, results mapped back through inner_global
# --------------------------------------------------------------------------- #
def _assignment_worker(rank, world, src, dst, n, assign, exchange):
    import torch.distributed as dist
    _install_stand_ins()
    a = th.from_numpy(assign)
    part = D.build_partition_from_assignment(th.from_numpy(src), th.from_numpy(dst), a, rank,
                                             num_parts=world, exchange=exchange, tau=3)
    own = part.inner_global
    assert th.equal(th.sort(own).values, th.nonzero(a == rank).flatten())
    xg = th.randn(n, 4, generator=th.Generator().manual_seed(3), dtype=th.float64)
    ref = _whole(src, dst, n, xg)[own]
    xi = xg[own].contiguous()
    out = D.aggregate_with_halo(xi, part) if exchange == "pull" else D.aggregate_hybrid(xi, part)
    assert th.allclose(out, ref, atol=1e-9)
    # every node is owned by exactly one rank
    counts = th.zeros(n, dtype=th.int64)
    counts[own] += 1
    dist.all_reduce(counts)
    assert bool((counts == 1).all())
    dist.barrier()


@pytest.mark.parametrize("world,exchange", [(4, "pull"), (8, "pull"), (8, "hybrid")])
def test_partition_from_any_assignment(world, exchange):
    """A scattered assignment (node v on part hash(v) % world, part 5 of 8 left empty)."""
    src, dst, n = powerlaw(3000, 40000, seed=30 + world)
    rng = np.random.default_rng(world)
    assign = rng.integers(0, world, n)
    if world == 8:
        assign[assign == 5] = 6
    run_world(_assignment_worker, world, (src, dst, n, assign, exchange))


# --------------------------------------------------------------------------- #
# flattened gradient all-reduce at world 8
# --------------------------------------------------------------------------- #
def _allreduce_worker(rank, world):
    import torch.distributed as dist
    ps = [th.nn.Parameter(th.zeros(3, 2)), th.nn.Parameter(th.zeros(5)), th.nn.Parameter(th.zeros(1))]
    ps[0].grad = th.full((3, 2), float(rank))
    ps[1].grad = th.arange(5, dtype=th.float32) * (rank + 1)
    # ps[2] has no gradient (a frozen parameter): skipped, the others still reduced
    D.allreduce_gradients(ps)
    mean_r = sum(range(world)) / world
    assert th.allclose(ps[0].grad, th.full((3, 2), mean_r))
    assert th.allclose(ps[1].grad, th.arange(5, dtype=th.float32) * (mean_r + 1))
    assert ps[2].grad is None
    dist.barrier()


def test_allreduce_gradients_world8():
    run_world(_allreduce_worker, 8, ())
