#!/usr/bin/env python3
"""Fused GAT kernels on the C3 Reddit-size graph (232,965 nodes, 114.6 M edges,
8 heads x 8), for rocprofv3 kernel traces and PMC passes: --reps forward and
backward launches each (kernel-level, no autograd)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch as th  # noqa: E402

from dgl import kernel as K  # noqa: E402
from bench_configs import chung_lu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks", default=None, help="DGLMI_GAT_BLOCKS (default: automatic)")
    args = ap.parse_args()
    if args.blocks is not None:
        os.environ["DGLMI_GAT_BLOCKS"] = args.blocks
    dev = "cuda:0"
    n, m, H, D = 232965, 114615892, 8, 8
    g = chung_lu(n, m, 0.4, 3, dev)
    gidx = g._graph.get_immutable_gidx(dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(3)
    ft = th.randn(n, H, D, device=dev, generator=gen)
    el = th.randn(n, H, device=dev, generator=gen)
    er = th.randn(n, H, device=dev, generator=gen)
    go = th.randn(n, H, D, device=dev, generator=gen)
    out = th.empty(n, H, D, device=dev)
    mx, sm = th.empty(n, H, device=dev), th.empty(n, H, device=dev)
    gft, gel, ger = th.empty_like(ft), th.empty_like(el), th.empty_like(er)
    th.cuda.synchronize()
    res = {"col_blocks": K.gat_col_blocks(gidx, ft)}
    for name, fn in (("fwd", lambda: K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm)),
                     ("bwd", lambda: K.fused_gat_backward(gidx, ft, el, er, 0.2, out, mx, sm, go,
                                                          gft, gel, ger))):
        fn()
        th.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.reps):
            fn()
        th.cuda.synchronize()
        res[name + "_ms"] = (time.perf_counter() - t) * 1e3 / args.reps
    res["checksum"] = float(out.double().sum()) + float(gft.double().sum())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
