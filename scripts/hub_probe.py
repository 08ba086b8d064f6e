#!/usr/bin/env python3
"""Mega-hub rows: one destination with millions of in-edges spans thousands of
chunks, and its carries are folded by k_chunk_fixup.  Times copy_u_sum (F = 64)
and the fused GAT forward on 20 M edges (a) spread uniformly over 1 M rows,
(b) all into row 0 (a star), (c) into 4 hubs; HIP-event medians.  One JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import dgl  # noqa: E402
import dgl.backend as B  # noqa: E402
from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def ktime(fn, steps=10):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    dev = "cuda:0"
    n, m, f = 1 << 20, 20_000_000, 64
    gen = th.Generator(device=dev).manual_seed(0)
    src = th.randint(0, n, (m,), generator=gen, device=dev, dtype=th.int32)
    x = th.rand(n, f, device=dev, generator=gen)
    res = {"nodes": n, "edges": m, "feat": f}
    cases = {
        "uniform": th.randint(0, n, (m,), generator=gen, device=dev, dtype=th.int32),
        "star": th.zeros(m, dtype=th.int32, device=dev),
        "four_hubs": (th.randint(0, 4, (m,), generator=gen, device=dev, dtype=th.int32) * 1000),
    }
    for name, dst in cases.items():
        log("%s: building CSRs" % name)
        gidx = device_block_gidx(n, n, src, dst)
        out = th.empty(n, f, device=dev)
        log("%s: copy_u_sum" % name)
        ms = ktime(lambda: K.copy_reduce("sum", gidx, 0, x, out))
        log("%s: copy_u_sum %.3f ms; checking" % (name, ms))
        if name == "uniform":
            ref = th.zeros(n, f, dtype=th.float64, device=dev).index_add_(0, dst.long(), x[src.long()].double())
        else:  # a few hub rows: per-hub reductions (fp64 atomics into one row crawl)
            ref = th.zeros(n, f, dtype=th.float64, device=dev)
            for h in th.unique(dst).tolist():
                ref[h] = x[src[dst == h].long()].double().sum(0)
        err = float(((out.double() - ref).abs().max() / ref.abs().max()).item())
        log("%s: fused GAT" % name)
        g = dgl.DGLGraph.from_device_coo(src, dst, n)
        ft = th.rand(n, 8, 8, device=dev, generator=gen)
        el = th.rand(n, 8, 1, device=dev, generator=gen)
        er = th.rand(n, 8, 1, device=dev, generator=gen)
        gat = ktime(lambda: B.fused_gat(g, ft, el, er, 0.2))
        res[name] = {"copy_u_sum_ms": ms, "rel_err": err, "fused_gat_fwd_ms": gat}
        print(name, res[name], file=sys.stderr, flush=True)
        del gidx, out, ref, g
        th.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
