#!/usr/bin/env python3
"""Is the C5 rehearsal graph (Chung-Lu 1 M / 16 M) and its label-propagation
partition the same on two builds in one process?  Prints which step differs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch as th  # noqa: E402


def main():
    from bench_configs import chung_lu
    from dgl import distributed as D
    dev = "cuda:0"
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 16_000_000
    res = {"n": n, "m": m}
    runs = []
    for _ in range(2):
        g = chung_lu(n, m, 0.5, 8, dev)
        src, dst = g._graph._device_only
        gidx = g._graph.get_immutable_gidx(dev)
        parts = [D.partition_labelprop(gidx, 2, rounds=24, slack=0.02)[0] for _ in range(2)]
        runs.append((src.clone(), dst.clone(), gidx.in_csr.indptr.clone(), gidx.in_csr.indices.clone(),
                     parts))
    (s0, d0, p0, i0, a0), (s1, d1, p1, i1, a1) = runs
    res["coo_equal"] = bool(th.equal(s0, s1) and th.equal(d0, d1))
    res["csr_equal"] = bool(th.equal(p0, p1) and th.equal(i0, i1))
    res["lp_equal_same_graph"] = bool(th.equal(a0[0], a0[1]))
    res["lp_equal_across_builds"] = bool(th.equal(a0[0], a1[0]))
    res["lp_diff_nodes"] = int((a0[0] != a0[1]).sum())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
