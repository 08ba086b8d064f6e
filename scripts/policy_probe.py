#!/usr/bin/env python3
"""Cache-policy probe for the M1 copy_u_sum gather: the hot-row threshold
(DGLMI_HOT_DEGREE) crossed with the load policy of marked (cold) and unmarked
rows (DGLMI_SPMM_POLICY, spmm_chunk.h var_pol: buffer loads with aux bits
sc0 = 1, nt = 2, sc1 = 16), HIP-event medians per launch; every variant is
checked bit-exact against the shipped launch.  --relabel also times the graph
with source ids renumbered by out-degree (hot rows packed at the front of X)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

# the policy / tuning variants live in the probe build (make -C dgl-hack_amd PROBES=1)
os.environ.setdefault("DGLMI_PROBES", "1")

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import bench  # noqa: E402
from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402

POLICIES = {0: "shipped (global, cold nt)", 1: "buf hot plain / cold nt", 2: "cold sc1",
            3: "cold sc0 sc1", 4: "cold nt sc1", 5: "cold sc0 nt", 6: "hot sc0 / cold nt",
            7: "hot sc1 / cold nt", 8: "buf all plain", 9: "buf all nt"}


def ktime(fn, steps=10):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def sweep(g, x, out, hots, pols, tag, res):
    ref = None
    for hot in hots:
        os.environ["DGLMI_HOT_DEGREE"] = str(hot)
        g._gather_cols = None
        g.MAX_COLD_SHARE = 1.0
        for pol in pols:
            os.environ["DGLMI_SPMM_POLICY"] = str(pol)
            t = ktime(lambda: K.copy_reduce("sum", g, 0, x, out))
            if ref is None:
                ref = out.clone()
            key = "%s_hot%d_pol%d" % (tag, hot, pol)
            res[key] = {"ms": t, "exact": bool(th.equal(out, ref)), "policy": POLICIES[pol]}
            ic, _ = g.gather_cols()
            if ic is not None:
                res[key]["cold_edge_share"] = float((ic < 0).float().mean())
            print(key, json.dumps(res[key]), flush=True)
    os.environ["DGLMI_SPMM_POLICY"] = "0"
    os.environ.pop("DGLMI_HOT_DEGREE", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hot", default="64,256,1024,4096")
    ap.add_argument("--pol", default="0,1,2,3,4,5,6,7,8,9")
    ap.add_argument("--relabel", action="store_true")
    ap.add_argument("--out", default="gpurun_out/policy_probe.json")
    args = ap.parse_args()
    dev = "cuda:0"
    hots = [int(h) for h in args.hot.split(",")]
    pols = [int(p) for p in args.pol.split(",")]
    n, n_dst, src, dst, x = bench.build_workload(1, 0, dev)
    res = {"nodes": n, "edges": int(src.shape[0])}
    out = th.empty(n_dst, bench.FEAT, device=dev)
    if args.relabel:
        deg = th.bincount(src.long(), minlength=n)
        order = th.argsort(deg, descending=True, stable=True)
        new_of = th.empty_like(order)
        new_of[order] = th.arange(n, device=dev)
        g2 = device_block_gidx(n, n_dst, new_of[src.long()].to(th.int32), dst)
        x2 = x[order].contiguous()
        del deg, new_of
        sweep(g2, x2, out, hots[:2], [0, 1], "relabel", res)
        o2 = out.clone()
        del g2, x2
    g = device_block_gidx(n, n_dst, src, dst)
    del src, dst
    sweep(g, x, out, hots, pols, "m1", res)
    if args.relabel:
        res["relabel_max_rel_diff"] = float((o2 - out).abs().max() / out.abs().max())
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
