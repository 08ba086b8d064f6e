#!/usr/bin/env python3
"""One C3 training step of GATConv (602 -> 8 x 8 heads, fused route, no dropout) on the
Reddit-size graph, repeated --steps times after --warmup: run it under
`rocprofv3 --kernel-trace --stats` to see where the step's time goes kernel by kernel
(the walks against the projections, el / er, torch elementwise work and allocations).
--composition: GATConv with use_fused = False (the reference's composition) instead.
--ab-logits: alternate the fused route's device el / er (gatconv.FUSED_ATTN_LOGITS) with
torch's multiply + sum, three rounds each, and print both series."""
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

from bench_configs import chung_lu  # noqa: E402
from dgl.nn.pytorch import GATConv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--composition", action="store_true")
    ap.add_argument("--ab-logits", action="store_true")
    args = ap.parse_args()
    dev = "cuda:0"
    g = chung_lu(232965, 114615892, 0.4, 3, dev)
    x = th.randn(232965, 602, device=dev)
    gat = GATConv(602, 8, 8).to(dev)
    gat.use_fused = not args.composition
    gat.train()

    def step():
        gat(g, x).sum().backward()
    def timed():
        for _ in range(args.warmup):
            step()
        th.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        th.cuda.synchronize()
        return (time.perf_counter() - t) * 1000 / args.steps
    if args.ab_logits:
        from dgl.nn.pytorch.conv import gatconv
        series = {"device_logits": [], "torch_logits": []}
        for _ in range(3):
            for flag, key in ((True, "device_logits"), (False, "torch_logits")):
                gatconv.FUSED_ATTN_LOGITS = flag
                series[key].append(timed())
        print(json.dumps({"route": "fused", "steps": args.steps, "ms_per_step": series}), flush=True)
        return
    print(json.dumps({"route": "composition" if args.composition else "fused", "steps": args.steps,
                      "ms_per_step": timed()}), flush=True)


if __name__ == "__main__":
    main()
