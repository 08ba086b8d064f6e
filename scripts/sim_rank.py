#!/usr/bin/env python3
"""Per-rank kernel time of the weak-scaling bench, simulated on one GPU.

Rank r of W sees the scale 23+log2(W) RMAT graph's in-edges of its row block.
Compares the SpMM over the replicated global X (global source ids) with the
same SpMM over a compacted [owned | halo] table (local source ids), the layout
of the halo partition."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import bench  # noqa: E402


def ktime(fn, steps=10):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    dev = "cuda:0"
    from dgl import kernel as K
    from dgl.graph_index import device_block_gidx
    n, n_dst, src, dst, x = bench.build_workload(args.world, args.rank, dev)
    lo = n * args.rank // args.world
    g = device_block_gidx(n, n_dst, src, dst)
    out = th.empty(n_dst, bench.FEAT, device=dev)
    t_rep = ktime(lambda: K.copy_reduce("sum", g, 0, x, out))
    # compacted: owned rows first, then the remote sources in ascending id order
    s = src.long()
    remote = (s < lo) | (s >= lo + n_dst)
    halo = th.unique(s[remote])
    local = th.where(remote, n_dst + th.searchsorted(halo, s), s - lo).to(th.int32)
    gl = device_block_gidx(n_dst + halo.shape[0], n_dst, local, dst)
    xl = th.cat([x[lo:lo + n_dst], x[halo]])
    out2 = th.empty_like(out)
    t_cmp = ktime(lambda: K.copy_reduce("sum", gl, 0, xl, out2))
    err = float((out - out2).abs().max())
    del gl, xl, out2, local
    # compacted and ordered by use count (hot source rows packed together: fewer
    # pages / DRAM rows touched by the re-read rows)
    uniq, inv, cnt = th.unique(s, return_inverse=True, return_counts=True)
    order = th.argsort(cnt, descending=True, stable=True)
    rank_of = th.empty_like(order)
    rank_of[order] = th.arange(order.shape[0], device=dev)
    lf = rank_of[inv].to(th.int32)
    gf = device_block_gidx(uniq.shape[0], n_dst, lf, dst)
    xf = x[uniq[order]]
    out3 = th.empty_like(out)
    t_freq = ktime(lambda: K.copy_reduce("sum", gf, 0, xf, out3))
    err = max(err, float((out - out3).abs().max()))
    print(json.dumps({"world": args.world, "rank": args.rank, "nodes": n, "local_edges": int(src.shape[0]),
                      "halo_rows": int(halo.shape[0]), "replicated_ms": t_rep, "compacted_ms": t_cmp,
                      "compacted_by_use_ms": t_freq, "distinct_sources": int(uniq.shape[0]),
                      "max_abs_diff": err}))


if __name__ == "__main__":
    main()
