#!/usr/bin/env python3
"""MFMA utilisation of the dense projections that bracket the aggregations.

Run under ``rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE`` once per
shape (``--shape``); each run issues ``--reps`` forward GEMMs (X W), then as many
input-gradient GEMMs (dY W^T), then as many weight-gradient products through
``dgl.backend.project``'s split-K path (the one GraphConv / GATConv /
RelGraphConv train with).  ``scripts/mfma_summary.py`` turns the counters into
utilisation = MFMA busy SIMD-cycles / (kernel cycles x 1024 SIMDs), and checks the
counter against the algorithmic FLOPs (fp32 MFMA: 64 FLOP per SIMD-cycle).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import torch as th  # noqa: E402

SHAPES = {"c1": (2708, 1433, 16), "c2": (169343, 128, 128), "c3": (232965, 602, 64),
          "c5": (5_000_000, 64, 256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", choices=sorted(SHAPES), required=True)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import dgl  # noqa: F401
    from dgl import backend as B
    m, k, n = SHAPES[args.shape]
    dev = "cuda:0"
    x = th.randn(m, k, device=dev)
    w = th.randn(k, n, device=dev)
    gy = th.randn(m, n, device=dev)
    th.cuda.synchronize()
    from dgl import kernel as K
    # the route B.project takes: the MFMA projection kernel where it applies (round 5),
    # hipBLASLt otherwise
    fwd = (lambda: K.project_mfma(x, w)) if K.project_mfma_ok(x, w) else (lambda: x @ w)
    wt = w.t()
    gx = (lambda: K.project_mfma(gy, wt)) if K.project_mfma_ok(gy, wt) else (lambda: gy @ wt)
    ops = [("fwd", fwd), ("grad_x", gx), ("grad_w", lambda: B.weight_grad(x, gy))]
    for _, fn in ops:
        for _ in range(args.reps):
            fn()
        th.cuda.synchronize()
    print(json.dumps({"shape": args.shape, "m": m, "k": k, "n": n, "reps": args.reps,
                      "ops": [o for o, _ in ops], "flops_per_gemm": 2.0 * m * k * n}))


if __name__ == "__main__":
    main()
