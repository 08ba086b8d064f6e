#!/usr/bin/env python3
"""Experiment: would cutting the C3 GAT aggregation into source blocks (one
launch per block of source rows, so the gathered ft/el slice shrinks towards
the 4 MiB per-XCD L2) cut the fabric traffic enough to pay for merging partial
(m, l, acc) rows?  Times k_gat_fwd over each block's sub-graph (all blocks
sequentially) against the whole graph; no merge is timed."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402
from bench_configs import chung_lu  # noqa: E402


def ktime(fn, steps=6):
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
    n, m, H, D = 232965, 114615892, 8, 8
    g = chung_lu(n, m, 0.4, 3, dev)
    src, dst = g._graph._device_only
    src, dst = src.to(dev), dst.to(dev)
    gidx = g._graph.get_immutable_gidx(th.device(dev))
    ft = th.randn(n, H, D, device=dev)
    el = th.randn(n, H, device=dev)
    er = th.randn(n, H, device=dev)
    out = th.empty(n, H, D, device=dev)
    mx, sm = th.empty(n, H, device=dev), th.empty(n, H, device=dev)
    res = {"whole_ms": ktime(lambda: K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm))}
    for nb in (2, 4, 8, 16):
        bounds = [n * b // nb for b in range(nb + 1)]
        subs = []
        for b in range(nb):
            sel = (src >= bounds[b]) & (src < bounds[b + 1])
            subs.append(device_block_gidx(n, n, src[sel], dst[sel]))
        tot = 0.0
        for sg in subs:
            tot += ktime(lambda: K.fused_gat_forward(sg, ft, el, er, 0.2, out, mx, sm))
        res["blocks%d_sum_ms" % nb] = tot
        del subs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
