#!/usr/bin/env python3
"""Kernel-level timing of copy_u_sum on the M1 graph (interleaved A/B rounds).

  python scripts/tune_spmm.py --mode sweep     # chunk sizes x rounds, HIP events
  python scripts/tune_spmm.py --mode single    # a few launches (for rocprofv3 --pmc)
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="sweep")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--chunks", default="64,128,256,512,1024")
    ap.add_argument("--feats", default="64")
    ap.add_argument("--variants", default="0")
    args = ap.parse_args()
    if args.mode != "single":
        # chunk sizes and variants are picked in the probe build (make -C dgl-hack_amd PROBES=1)
        os.environ.setdefault("DGLMI_PROBES", "1")
    dev = "cuda:0"
    th.cuda.set_device(0)
    from dgl import kernel as K
    n, n_dst, src, dst, x = bench.build_workload(1, 0, dev)
    gidx, _ = bench.make_local_graph(n, n_dst, src, dst, dev)
    m = src.shape[0]
    del src, dst
    res = {}
    feats = [int(f) for f in args.feats.split(",")]
    chunks = [int(c) for c in args.chunks.split(",")]
    if args.mode == "single":
        out = th.empty(n_dst, 64, device=dev)
        for _ in range(args.steps):
            K.copy_reduce("sum", gidx, 0, x, out)
        th.cuda.synchronize()
        return
    xs = {f: (x if f == 64 else th.rand(n, f, device=dev)) for f in feats}
    outs = {f: th.empty(n_dst, f, device=dev) for f in feats}
    variants = [int(v) for v in args.variants.split(",")]
    for r in range(args.rounds):
        for f in feats:
            for c in chunks:
              for var in variants:
                os.environ["DGLMI_CHUNK_EDGES"] = str(c)
                os.environ["DGLMI_SPMM_VARIANT"] = str(var)
                K.copy_reduce("sum", gidx, 0, xs[f], outs[f])
                evs = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True))
                       for _ in range(args.steps)]
                for a, b in evs:
                    a.record()
                    K.copy_reduce("sum", gidx, 0, xs[f], outs[f])
                    b.record()
                th.cuda.synchronize()
                ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
                res.setdefault("F%d_K%d_V%d" % (f, c, var), []).append(ms)
    os.environ.pop("DGLMI_CHUNK_EDGES", None)
    os.environ.pop("DGLMI_SPMM_VARIANT", None)
    summary = {}
    for k, v in res.items():
        f = int(k.split("_")[0][1:])
        ms = float(np.median(v))
        alg = 4 * (n_dst + 1) + 4 * m + 4 * f * m + 4 * f * n_dst
        summary[k] = {"ms": ms, "min_ms": float(np.min(v)), "alg_GBps": alg / ms / 1e6,
                      "Gedges_s": m / ms / 1e6}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
