#!/usr/bin/env python3
"""C5 RelGraphConv (4 relations, basis, 64 -> 64, self-loop, bias, per-edge norm) on
the Chung-Lu graph of scripts/bench_configs.py: a few forward and forward + backward
calls for rocprofv3 kernel statistics, plus HIP-event medians of both (--time)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def main():
    from bench_configs import chung_lu
    from dgl.nn.pytorch import RelGraphConv
    dev = "cuda:0"
    n, m, R, f = 5_000_000, 80_000_000, 4, 64
    g = chung_lu(n, m, 0.5, 8, dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), generator=gen, device=dev)
    src, dst = g._graph._device_only
    indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
    norm = (1.0 / indeg)[dst.long()].reshape(m, 1)
    x = th.randn(n, f, device=dev, requires_grad=True)
    conv = RelGraphConv(f, f, R, "basis", num_bases=R, self_loop=True).to(dev)
    if "--unfused" in sys.argv:
        conv.use_fused = False

    def fwd():
        with th.no_grad():
            conv(g, x, et, norm)

    def fwd_bwd():
        conv(g, x, et, norm).sum().backward()
    res = {}
    for name, fn in (("fwd", fwd), ("fwd_bwd", fwd_bwd)):
        for _ in range(2):
            fn()
        ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        th.cuda.synchronize()
        res[name + "_ms"] = float(np.median([a.elapsed_time(b) for a, b in ev]))
    res["fused"] = conv.use_fused
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
