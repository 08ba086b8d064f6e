#!/usr/bin/env python3
"""Probe: per-edge kernel item order (edge-id vs in-CSR) on a dense-ish graph
(C3 Reddit-size, average in-degree 492) for node-only operands."""
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
g = chung_lu(n, m, 0.4, 3, dev)
gidx = g._graph.get_immutable_gidx(dev)
res = {}
for name, op, shape in (("u_dot_v_8x8", "dot", (8, 8)), ("u_add_v_8", "add", (8,)),
                        ("u_dot_v_64", "dot", (64,))):
    a = th.rand((n,) + shape, device=dev)
    b = th.rand((n,) + shape, device=dev)
    for order in ("coo", "csr"):
        dgl.kernel.set_sddmm_order(order)
        res["%s_%s_ms" % (name, order)] = timeit(
            lambda: dgl.backend.binary_reduce("none", op, gidx, 0, 1, a, b, m), 10, 3)
    dgl.kernel.set_sddmm_order("auto")
print(json.dumps(res))
