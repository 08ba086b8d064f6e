#!/usr/bin/env python3
"""Partition quality and cost on C4 (10 M nodes / 200 M edges RMAT, bench.c4_workload):
contiguous id blocks (the previous planner: a random partition, ids are permuted)
vs the device label propagation (dgl.distributed.partition_labelprop) after R
rounds, for k = 2, 4, 8 -- cut fraction, halo rows (rows a layer's all-to-all-v
moves), edge balance, partitioner time.  --ldg also runs the host LDG
(DGLMIPartitionLDG) on a scale-20 RMAT for a quality reference."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import bench  # noqa: E402
from dgl import distributed as D  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402


def summary(st, n_edges):
    e = np.array(st["edges"], np.float64)
    return {"cut_fraction": st["cut_edges"] / n_edges, "halo_rows_total": int(sum(st["halo_rows"])),
            "halo_rows_max": int(max(st["halo_rows"])), "edge_imbalance": float(e.max() / e.mean()),
            "halo_rows": st["halo_rows"], "edges": st["edges"]}


SLACK = 0.05


def probe(src, dst, n, ks, rounds_list, tag, out):
    gidx = device_block_gidx(n, n, src, dst)
    m = int(src.shape[0])
    w = (gidx.in_csr.degrees() + 1).to(th.int32)
    for k in ks:
        ct = D.contiguous_parts_device(w, k)
        out["%s_k%d_contiguous" % (tag, k)] = summary(D.partition_stats(src, dst, ct, k), m)
        print(tag, k, "contiguous", json.dumps(out["%s_k%d_contiguous" % (tag, k)])[:200], flush=True)
        for r in rounds_list:
            th.cuda.synchronize()
            t0 = time.time()
            a, info = D.partition_labelprop(gidx, k, rounds=r, slack=SLACK)
            th.cuda.synchronize()
            dt = time.time() - t0
            rec = summary(D.partition_stats(src, dst, a, k), m)
            rec["seconds"] = dt
            rec["loads"] = info["loads"]
            out["%s_k%d_lp%d" % (tag, k, r)] = rec
            print(tag, k, "lp", r, "%.2fs" % dt, json.dumps(rec)[:200], flush=True)
    return gidx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", default="8,24,48")
    ap.add_argument("--ks", default="2,4,8")
    ap.add_argument("--ldg", action="store_true")
    ap.add_argument("--slack", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/partition_probe.json")
    args = ap.parse_args()
    dev = "cuda:0"
    rounds = [int(r) for r in args.rounds.split(",")]
    global SLACK
    SLACK = args.slack
    ks = [int(k) for k in args.ks.split(",")]
    out = {}
    t0 = time.time()
    src, dst, _ = bench.c4_workload(dev)
    th.cuda.synchronize()
    out["c4_generate_s"] = time.time() - t0
    probe(src, dst, bench.C4_NODES, ks, rounds, "c4", out)
    del src, dst
    if args.ldg:
        s, d = bench.rmat_edges(20, 16 << 20, seed=5, device=dev)
        n = 1 << 20
        gp = th.Generator(device=dev)
        gp.manual_seed(5)
        perm = th.randperm(n, generator=gp, device=dev).to(th.int32)
        s, d = perm[s.long()].contiguous(), perm[d.long()].contiguous()
        probe(s, d, n, [8], rounds, "rmat20", out)
        t0 = time.time()
        a = D.partition_ldg(n, s.cpu().numpy(), d.cpu().numpy(), 8)
        dt = time.time() - t0
        rec = summary(D.partition_stats(s, d, th.from_numpy(a).to(dev), 8), int(s.shape[0]))
        rec["seconds"] = dt
        out["rmat20_k8_ldg_host"] = rec
        print("rmat20 8 ldg %.2fs" % dt, json.dumps(rec)[:200], flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
