#!/usr/bin/env python3
"""Full-graph training of the BASELINE GAT and R-GCN configs partitioned over
the GPUs of one node:

  --model gat   C3: GATConv 8 heads x 8 on a Reddit-size graph (232,965 nodes,
                114.6 M edges, 602 input features), 2 layers
  --model rgcn  C5: RelGraphConv, 4 relations, basis, on 5 M nodes / 80 M typed
                edges, 64 -> 64 -> 16, per-edge norm 1 / in-degree

  python examples/dist_train.py --model rgcn                        # 1 GPU
  torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/dist_train.py --model rgcn

One process per GPU.  Every rank draws the same synthetic graph on its GPU
(Chung-Lu power law, seeded; the datasets need downloads), partitions it with
the device label propagation (``dgl.distributed.partition_labelprop``, the
METIS stand-in), owns its part's nodes and all their in-edges, plans its halo
on the device (``build_partition_from_assignment``) and trains with
``DistGATConv`` / ``DistRelGraphConv``: one all-to-all-v per layer and
direction for the halo rows (RCCL over xGMI), the fused GAT kernel or the
typed gather on the local block, one flattened gradient all-reduce per step.
The partition-parallel modules equal the whole-graph ones
(``tests/test_distributed_gpu.py``).

Prints one JSON line (rank 0): epoch time (max over ranks), halo sizes, loss.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dgl-hack_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch as th  # noqa: E402

CONFIGS = {
    "gat": dict(nodes=232_965, edges=114_615_892, alpha=0.4, feat=602, hidden=8, heads=8,
                classes=41, seed=3),
    "rgcn": dict(nodes=5_000_000, edges=80_000_000, alpha=0.5, feat=64, hidden=64, rels=4,
                 classes=16, seed=8),
}


def chung_lu(n, m, alpha, seed, device):
    """Power-law edge list (same draw as scripts/bench_configs.py), identical on
    every rank."""
    from dgl.data.synthetic import chung_lu_edges
    return chung_lu_edges(n, m, alpha, seed, device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=sorted(CONFIGS), default="rgcn")
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the config's size")
    ap.add_argument("--dist-backend", default="nccl")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (rehearsal)")
    ap.add_argument("--no-fused", action="store_true",
                    help="rgcn: the GEMM + typed-gather path instead of the fused R-GCN kernels")
    args = ap.parse_args()
    cfg = CONFIGS[args.model]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    th.cuda.set_device(local)
    dev = "cuda:%d" % local
    dist = None
    cdev = dev
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=th.device(dev))
        else:
            dist.init_process_group(args.dist_backend)
            cdev = "cpu"
    from dgl import distributed as D

    n = int(cfg["nodes"] * args.scale)
    m = int(cfg["edges"] * args.scale)
    t0 = time.time()
    src, dst = chung_lu(n, m, cfg["alpha"], cfg["seed"], dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(cfg["seed"] + 1)
    # device label propagation (the METIS stand-in), identical on every rank
    if world > 1:
        from dgl.graph_index import device_block_gidx
        assign, _ = D.partition_labelprop(device_block_gidx(n, n, src, dst), world)
    else:
        assign = th.zeros(n, dtype=th.int32, device=dev)
    sel = assign[dst.long()] == rank   # local edge order = build_partition_from_assignment's
    if args.model == "rgcn":
        et = th.randint(0, cfg["rels"], (m,), generator=gen, device=dev)
        indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
        et_l = et[sel]
        norm_l = (1.0 / indeg)[dst[sel].long()].view(-1, 1)
        del et, indeg
    part = D.build_partition_from_assignment(src, dst, assign, rank, None, world)
    del src, dst, sel
    inner = part.inner_global
    n_own = part.n_inner
    part.gidx()
    part.local_graph()
    th.cuda.synchronize()
    t_setup = time.time() - t0

    gx = th.Generator(device=dev)
    gx.manual_seed(7)
    x = th.randn(n, cfg["feat"], generator=gx, device=dev)[inner].contiguous()
    y = th.randint(0, cfg["classes"], (n,), generator=gx, device=dev)[inner]
    th.manual_seed(0)
    if args.model == "gat":
        l1 = D.DistGATConv(cfg["feat"], cfg["hidden"], cfg["heads"], activation=th.nn.functional.elu)
        l2 = D.DistGATConv(cfg["hidden"] * cfg["heads"], cfg["classes"], 1)

        def forward():
            h = l1(part, x).reshape(n_own, -1)
            return l2(part, h).mean(1)
    else:
        l1 = D.DistRelGraphConv(cfg["feat"], cfg["hidden"], cfg["rels"], "basis",
                                num_bases=cfg["rels"], self_loop=True, activation=th.relu)
        l2 = D.DistRelGraphConv(cfg["hidden"], cfg["classes"], cfg["rels"], "basis",
                                num_bases=cfg["rels"], self_loop=True)
        if args.no_fused:
            l1.conv.use_fused = l2.conv.use_fused = False

        def forward():
            return l2(part, l1(part, x, et_l, norm_l), et_l, norm_l)
    l1, l2 = l1.to(dev), l2.to(dev)
    params = list(l1.parameters()) + list(l2.parameters())
    opt = th.optim.Adam(params, lr=0.01)

    def epoch():
        opt.zero_grad()
        logp = th.log_softmax(forward(), dim=1)
        loss = -logp.gather(1, y.view(-1, 1)).sum() / n
        loss.backward()
        D.allreduce_gradients(params, average=False)
        opt.step()
        return loss

    for _ in range(args.warmup):
        epoch()
    if dist is not None:
        dist.barrier()
    th.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.epochs):
        loss = epoch()
    th.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t
    stats = th.tensor([el, float(part.n_halo), float(part.number_of_edges())], dtype=th.float64,
                      device=cdev)
    if dist is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats.clone()
        dist.all_reduce(tot)
        el, halo_max, halo_rows, edges = float(mx[0]), int(mx[1]), int(tot[1]), int(tot[2])
        lsum = loss.detach().to(cdev).reshape(1)
        dist.all_reduce(lsum)
        loss_v = float(lsum)
    else:
        halo_max = halo_rows = int(stats[1])
        edges = int(stats[2])
        loss_v = float(loss.detach())
    ms = el * 1000 / args.epochs
    if rank == 0:
        print(json.dumps({
            "config": ("C3 GAT 8x8, 2 layers" if args.model == "gat" else
                       "C5 R-GCN 4 relations basis, 2 layers") +
                      ", %d nodes / %d edges (Chung-Lu)" % (n, m),
            "n_gpus": world, "epoch_ms": ms, "setup_s": t_setup, "edges": edges,
            "halo_rows_total": halo_rows, "max_halo_rows_per_rank": halo_max, "loss": loss_v,
            "partition": "contiguous id ranges (permuted ids), device halo plan",
            "collectives": dist.get_backend() if dist is not None else "none"}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
