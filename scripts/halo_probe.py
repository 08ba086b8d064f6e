#!/usr/bin/env python3
"""How many rows must a C4 layer move at k = 8?  For a node assignment, the
pull-only exchange moves every distinct (remote source, destination part) row;
a hybrid exchange may instead push the partial sum of a destination v over the
sources a part p holds for it (one row per (v, p)) when that replaces >= tau
pulled rows' worth of edges.  Reports pull-only, push-only and greedy hybrid row
counts for: contiguous ids (random), device label propagation, and -- for
scale only -- the RMAT generator's own id-bit blocks (not available to a real
partitioner: it reads the generator's id map)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import torch as th  # noqa: E402

import bench  # noqa: E402
from dgl import distributed as D  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402


def volumes(src, dst, a, k, n, taus):
    s, d = src.long(), dst.long()
    ps, pd = a[s].long(), a[d].long()
    x = ps != pd
    s, d, ps, pd = s[x], d[x], ps[x], pd[x]
    pairs = th.unique(s * n + d)                  # distinct cross (u, v)
    u, v = pairs // n, pairs % n
    pu, pv = a[u].long(), a[v].long()
    pull = int(th.unique(u * k + pv).numel())     # rows (u -> part of v)
    vp, cnt = th.unique(v * k + pu, return_counts=True)
    push = int(vp.numel())                        # partials (v <- part of u)
    res = {"cross_edges": int(x.sum()), "pull_rows": pull, "push_rows": push, "hybrid": {}}
    c_of_pair = cnt[th.searchsorted(vp, v * k + pu)]
    # per-part SpMM work of the hybrid step at tau = 8 (what bench's
    # spmm_edges_per_rank counts): owned block + push block + receive block
    # (edges of pulled rows, one entry per incoming partial row)
    pos = th.searchsorted(vp, d * k + ps)            # (v, part of u) of every cut edge
    pushed_e = cnt[pos] >= 8
    a_all = a.long()
    a_src, a_dst = a_all[src.long()], a_all[dst.long()]
    own = th.bincount(a_dst[a_src == a_dst], minlength=k)
    push_w = th.bincount(ps[pushed_e], minlength=k)
    partials_in = th.bincount(a_all[vp[cnt >= 8] // k], minlength=k)
    recv_w = th.bincount(pd[~pushed_e], minlength=k) + partials_in
    work = (own + push_w + recv_w).tolist()
    res["hybrid_tau8_work_per_part"] = work
    res["hybrid_tau8_work_imbalance"] = max(work) / (sum(work) / k)
    res["edges_per_part"] = th.bincount(a_dst, minlength=k).tolist()
    for t in taus:
        pushed = c_of_pair >= t
        n_push = int((cnt >= t).sum())
        rest = th.unique(u[~pushed] * k + pv[~pushed]).numel()
        res["hybrid"][str(t)] = {"push_rows": n_push, "pull_rows": int(rest), "total": n_push + int(rest)}
    # edge-level rule: cover each cut edge by its heavier endpoint in the bipartite
    # cut graph between the two parts (push v when c(v, p) > d(u, q), d = distinct
    # destinations of u on q), a vertex-cover heuristic
    up, dcnt = th.unique(u * k + pv, return_counts=True)
    d_of = dcnt[th.searchsorted(up, u * k + pv)]
    for name, push in (("cover_gt", c_of_pair > d_of), ("cover_ge", c_of_pair >= d_of)):
        n_push = int(th.unique((v * k + pu)[push]).numel())
        n_pull = int(th.unique((u * k + pv)[~push]).numel())
        res["hybrid"][name] = {"push_rows": n_push, "pull_rows": n_pull, "total": n_push + n_pull}
    return res


def main():
    dev = "cuda:0"
    k, n = int(os.environ.get("K", "8")), bench.C4_NODES
    src, dst, perm = bench.c4_workload(dev, return_perm=True)
    taus = [2, 3, 4, 8, 16]
    out = {}
    g = device_block_gidx(n, n, src, dst)
    w = (g.in_csr.degrees() + 1).to(th.int32)
    ct = D.contiguous_parts_device(w, k).long()
    out["contiguous"] = volumes(src, dst, ct, k, n, taus)
    print("contiguous", json.dumps(out["contiguous"]), flush=True)
    lp, _ = D.partition_labelprop(g, k, rounds=24, slack=float(os.environ.get("SLACK", "0.02")))
    out["labelprop"] = volumes(src, dst, lp.long(), k, n, taus)
    print("labelprop", json.dumps(out["labelprop"]), flush=True)
    inv = th.empty_like(perm.long())
    inv[perm.long()] = th.arange(n, device=dev)
    bits = inv * k // n                           # 8 equal ranges of generator ids
    out["generator_bits"] = volumes(src, dst, bits, k, n, taus)
    print("generator_bits", json.dumps(out["generator_bits"]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/halo_probe_k%d.json" % k, "w"), indent=1)


if __name__ == "__main__":
    main()
