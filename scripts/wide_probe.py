#!/usr/bin/env python3
"""copy_u_sum (and copy_u_max) forward / backward kernel time vs feature width on the Reddit-size
graph (232,965 nodes / 114,615,892 edges): wide rows, including widths that are
not a multiple of 4 floats (F_in = 602 of Reddit)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch as th  # noqa: E402

import dgl  # noqa: E402
from bench_configs import chung_lu, timeit  # noqa: E402

dev = "cuda:0"
n, m = 232965, 114615892
g = chung_lu(n, m, 0.6, 3, dev)
gidx = g._graph.get_immutable_gidx(dev)
res = {"graph": "Reddit-size Chung-Lu", "nodes": n, "edges": m}
for f in [int(a) for a in (sys.argv[1] if len(sys.argv) > 1 else "64,128,256,600,602").split(",")]:
    x = th.randn(n, f, device=dev)
    out = th.empty(n, f, device=dev)
    gx = th.empty_like(x)
    ms_f = timeit(lambda: dgl.kernel.copy_reduce("sum", gidx, 0, x, out), 3, 1)
    ms_b = timeit(lambda: dgl.kernel.backward_copy_reduce("sum", gidx, 0, x, out, out, gx), 3, 1)
    dgl.kernel.copy_reduce("max", gidx, 0, x, out)
    ms_mf = timeit(lambda: dgl.kernel.copy_reduce("max", gidx, 0, x, out), 3, 1)
    ms_mb = timeit(lambda: dgl.kernel.backward_copy_reduce("max", gidx, 0, x, out, out, gx), 3, 1)
    alg = 4 * f * m
    res["F%d" % f] = {"fwd_ms": ms_f, "bwd_ms": ms_b, "fwd_gather_GBps": alg / ms_f / 1e6,
                      "bwd_gather_GBps": alg / ms_b / 1e6, "max_fwd_ms": ms_mf,
                      "max_bwd_ms": ms_mb}
    print(json.dumps({"F": f, **res["F%d" % f]}), flush=True)
    del x, out, gx
print(json.dumps(res))
