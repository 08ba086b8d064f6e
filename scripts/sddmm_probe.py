#!/usr/bin/env python3
"""Narrow g-SDDMM (one lane per edge) on M1 (RMAT scale 23, 100 M edges,
edge-id order): u_add_v with H = 8 / 4 / 1 values per node row, time and a
checksum over the output's raw bits.  profiles/r02_sddmm_variants.jsonl holds the
round-2 sweep of kernel variants run through it (streaming output stores,
non-temporal item-stream loads, two edges per lane; all within +-2 %, dropped):
the time tracks the number of random line requests (two per edge), not bytes --
H = 1 takes 2.9 ms, H = 8 3.6 ms."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--heads", default="8,4,1")
    ap.add_argument("--once", action="store_true", help="one launch per H (profiler runs)")
    args = ap.parse_args()
    import bench
    import dgl
    dev = "cuda:0"
    n, _, src, dst, _ = bench.build_workload(1, 0, dev)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    gidx = g._graph.get_immutable_gidx(dev)
    m = int(src.shape[0])
    del src, dst
    res = {"edges": m}
    gen = th.Generator(device=dev)
    gen.manual_seed(3)
    for h in [int(x) for x in args.heads.split(",")]:
        el = th.rand(n, h, device=dev, generator=gen)
        er = th.rand(n, h, device=dev, generator=gen)
        fn = lambda: dgl.backend.binary_reduce("none", "add", gidx, 0, 1, el, er, m)
        if args.once:
            fn()
            th.cuda.synchronize()
            continue
        ms = ktime(fn)
        out = fn()
        bits = out.contiguous().view(th.int32).reshape(-1).long()
        w = th.arange(1, bits.numel() + 1, device=dev) % 1000003
        res["H%d" % h] = {"ms": ms, "alg_GBps": (8 + 12 * h) * m / ms / 1e6,
                          "checksum": int(((bits & 0xFFFFFFFF) * w % 2147483647).sum().item())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
