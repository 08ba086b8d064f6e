#!/usr/bin/env python3
"""How much of M1's copy_u_sum time is the permuted ids' lack of locality?

Times the forward launch (HIP events, median of 10) on the same 100 M RMAT edges
under four node numberings: (a) the bench's random permutation, (b) the RMAT
generator's own ids (the locality the recursion builds in: the ceiling any
reordering could recover), (c) Cuthill-McKee-style BFS order from the highest-
degree node on the permuted graph (a reordering the library could compute on
the device), (d) nodes sorted by total degree (hubs first).  Prints one JSON."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import bench  # noqa: E402
from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402


def ktime(fn, steps=10):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def bfs_order(n, src, dst):
    """Level-synchronous BFS over the symmetrised graph; inside a level nodes are
    ordered by the position of their first-discovering parent (Cuthill-McKee
    without the degree tie-break).  Unreached nodes follow in id order."""
    dev = src.device
    s = th.cat([src, dst]).long()
    d = th.cat([dst, src]).long()
    key, perm = th.sort(s, stable=True)
    nbr = d[perm]
    del perm, d
    indptr = th.zeros(n + 1, dtype=th.long, device=dev)
    indptr[1:] = th.cumsum(th.bincount(key, minlength=n), 0)
    del key, s
    deg = indptr[1:] - indptr[:-1]
    pos = th.full((n,), -1, dtype=th.long, device=dev)
    root = int(th.argmax(deg).item())
    pos[root] = 0
    frontier = th.tensor([root], device=dev)
    placed = 1
    levels = 0
    while frontier.numel():
        levels += 1
        beg, cnt = indptr[frontier], deg[frontier]
        tot = int(cnt.sum().item())
        if tot == 0:
            break
        seg = th.repeat_interleave(th.arange(frontier.numel(), device=dev), cnt)
        off = th.arange(tot, device=dev) - th.repeat_interleave(th.cumsum(cnt, 0) - cnt, cnt)
        cand = nbr[beg[seg] + off]
        ppos = pos[frontier][seg]
        new = pos[cand] < 0
        cand, ppos = cand[new], ppos[new]
        best = th.full((n,), 1 << 62, dtype=th.long, device=dev)
        best.scatter_reduce_(0, cand, ppos, reduce="amin")
        nodes = th.nonzero(best < (1 << 62)).squeeze(1)
        order = th.argsort(best[nodes] * n + nodes)
        nodes = nodes[order]
        pos[nodes] = th.arange(placed, placed + nodes.numel(), device=dev)
        placed += nodes.numel()
        frontier = nodes
    rest = th.nonzero(pos < 0).squeeze(1)
    pos[rest] = th.arange(placed, placed + rest.numel(), device=dev)
    return pos.to(th.int32), levels


def run(name, n, src, dst, res, extra=None):
    g = device_block_gidx(n, n, src, dst)
    x = th.rand(n, bench.FEAT, device=src.device)
    out = th.empty(n, bench.FEAT, device=src.device)
    ms = ktime(lambda: K.copy_reduce("sum", g, 0, x, out))
    res[name] = dict(ms=ms, **(extra or {}))
    print(name, res[name], file=sys.stderr, flush=True)
    del g, x, out
    th.cuda.empty_cache()


def main():
    dev = "cuda:0"
    n = 1 << bench.SCALE
    src0, dst0 = bench.rmat_edges(bench.SCALE, bench.EDGES_PER_GPU, seed=1234, device=dev)
    gp = th.Generator(device=dev)
    gp.manual_seed(1)
    perm = th.randperm(n, generator=gp, device=dev).to(th.int32)
    src, dst = perm[src0.long()], perm[dst0.long()]
    del perm
    res = {"nodes": n, "edges": int(src.numel()), "feat": bench.FEAT}
    run("a_permuted", n, src, dst, res)
    run("b_generator_ids", n, src0, dst0, res)
    del src0, dst0
    th.cuda.synchronize()
    t0 = time.time()
    pos, levels = bfs_order(n, src, dst)
    th.cuda.synchronize()
    run("c_bfs_order", n, pos[src.long()], pos[dst.long()], res,
        {"order_s": time.time() - t0, "levels": levels})
    deg = th.bincount(src.long(), minlength=n) + th.bincount(dst.long(), minlength=n)
    rank = th.empty(n, dtype=th.int32, device=dev)
    rank[th.argsort(deg, descending=True, stable=True)] = th.arange(n, dtype=th.int32, device=dev)
    run("d_degree_sorted", n, rank[src.long()], rank[dst.long()], res)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
