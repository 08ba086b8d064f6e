#!/usr/bin/env python3
"""Cold-row hints (DGLMIGraph.{in,out}_gather_cols) on the M1 workload: copy_u_sum
forward (in-CSR) and its source gradient (out-CSR) with the hot threshold swept
(DGLMI_HOT_DEGREE; 0 = no hints), HIP-event medians per launch, results checked
bit-exact against the unhinted launch.  --world W times rank 0's graph of the
W-GPU weak-scaling workload."""
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
from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402


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
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--hot", default="0,16,32,64,128,256,0")
    args = ap.parse_args()
    dev = "cuda:0"
    n, n_dst, src, dst, x = bench.build_workload(args.world, 0, dev)
    g = device_block_gidx(n, n_dst, src, dst)
    del src, dst
    out = th.empty(n_dst, bench.FEAT, device=dev)
    gx = th.empty_like(x)
    go = th.randn(n_dst, bench.FEAT, device=dev)
    ref = gref = None
    res = {"world": args.world, "nodes": n, "edges": g.in_csr.nnz}
    for i, hot in enumerate(args.hot.split(",")):
        os.environ["DGLMI_HOT_DEGREE"] = hot
        g._gather_cols = None
        fwd = ktime(lambda: K.copy_reduce("sum", g, 0, x, out))
        bwd = ktime(lambda: K.backward_copy_reduce("sum", g, 0, x, out, go, gx))
        if ref is None:
            ref, gref = out.clone(), gx.clone()
        key = "hot%s_%d" % (hot, i)
        res[key + "_fwd_ms"] = fwd
        res[key + "_bwd_ms"] = bwd
        res[key + "_exact"] = bool(th.equal(out, ref)) and bool(th.equal(gx, gref))
        ic, oc = g.gather_cols()
        if ic is not None:
            res[key + "_cold_edge_share"] = float((ic < 0).float().mean())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
