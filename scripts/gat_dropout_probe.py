#!/usr/bin/env python3
"""C3-size fused GAT (232,965 nodes / 114.6 M edges, 8 x 8) forward + backward with and
without attention dropout (p = 0.6): HIP-event medians of each call, for rocprofv3
kernel statistics of the dropout path's cost (which walk grows)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def ktime(fn, steps=5):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    from bench_configs import chung_lu
    import dgl.backend as B
    dev = "cuda:0"
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.4, 3, dev)
    gen = th.Generator(device=dev).manual_seed(1)
    ft = th.randn(n, 8, 8, device=dev, generator=gen).requires_grad_()
    el = th.randn(n, 8, 1, device=dev, generator=gen).requires_grad_()
    er = th.randn(n, 8, 1, device=dev, generator=gen).requires_grad_()
    go = th.randn(n, 8, 8, device=dev, generator=gen)
    res = {}
    for p in (0.0, 0.6):
        def fwd():
            with th.no_grad():
                B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=5)

        def fwd_bwd():
            th.autograd.grad(B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=5), (ft, el, er), go)
        res["p%.1f_fwd_ms" % p] = ktime(fwd)
        res["p%.1f_fwd_bwd_ms" % p] = ktime(fwd_bwd)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
