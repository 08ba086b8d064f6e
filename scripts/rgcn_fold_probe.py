#!/usr/bin/env python3
"""R-GCN layer-1 backward with the weight gradient folded into the walk
(DGLMI_RGCN_FOLD=1, hack_kernels.hip k_rgcn_bwd_fold) against the round-4 backward (G_t
table + hidden^T . gy GEMM): RelGraphConv (basis, 64 -> 64, self-loop) on the C5
Chung-Lu graph with R relations (argv: R, default 4), forward + backward HIP-event
medians both ways and the largest gradient differences between them."""
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
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n, m, f = (int(sys.argv[2]), int(sys.argv[3]), 64) if len(sys.argv) > 3 else (5_000_000, 80_000_000, 64)
    g = chung_lu(n, m, 0.5, 8, dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), generator=gen, device=dev)
    src, dst = g._graph._device_only
    indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
    norm = (1.0 / indeg)[dst.long()].reshape(m, 1)
    x = th.randn(n, f, device=dev, requires_grad=True)
    go = th.randn(n, f, device=dev, generator=gen)
    th.manual_seed(0)
    conv = RelGraphConv(f, f, R, "basis", num_bases=R, self_loop=True).to(dev)
    params = [x] + list(conv.parameters())
    res = {"R": R, "nodes": n, "edges": m}
    grads = {}
    for fold in ("0", "1"):
        os.environ["DGLMI_RGCN_FOLD"] = fold

        def fwd_bwd():
            return th.autograd.grad(conv(g, x, et, norm), params, go)
        grads[fold] = fwd_bwd()
        fwd_bwd()
        ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record()
            fwd_bwd()
            b.record()
        th.cuda.synchronize()
        res["fold%s_fwd_bwd_ms" % fold] = float(np.median([a.elapsed_time(b) for a, b in ev]))
    worst = 0.0
    for a, b in zip(grads["1"], grads["0"]):
        worst = max(worst, float((a - b).abs().max()) / (1e-3 + 1e-4 * float(b.abs().max())))
    res["worst_err_over_bound"] = worst
    print(json.dumps(res), flush=True)
    if worst > 1.0:
        raise SystemExit("folded backward differs from the G_t + GEMM backward")


if __name__ == "__main__":
    main()
