#!/usr/bin/env python3
"""Would aggregating before the relation transform pay on C5 (5 M nodes, 80 M
edges, 4 relations, 64 features)?  Times the load-balanced typed gather of the
layer-1 forward as shipped (rows of Y = X W_cat, a 5.1 GB table, into N rows)
against the same gather over X (a 1.3 GB table) into N * R rows (dst-major
v * R + t, and relation-major t * N + v), norm streamed in walk order.  HIP-event
medians."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

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
    dev = "cuda:0"
    n, m, R, F = 5_000_000, 80_000_000, 4, 64
    g0 = th.Generator(device=dev)
    g0.manual_seed(8)
    src = th.randint(0, n, (m,), device=dev, generator=g0, dtype=th.int32)
    dst = th.randint(0, n, (m,), device=dev, generator=g0, dtype=th.int32)
    et = th.randint(0, R, (m,), device=dev, generator=g0, dtype=th.int32)
    norm = th.rand(m, 1, device=dev)
    res = {"config": "C5 typed gathers, 5M nodes / 80M edges / 4 relations / F=64"}
    cases = {
        "shipped_Y_table_to_N_rows": (n * R, n, src * R + et, dst),
        "X_table_to_NR_rows_dst_major": (n, n * R, src, dst * R + et),
        "X_table_to_NR_rows_rel_major": (n, n * R, src, et * n + dst),
    }
    for name, (ns, nd, s, d) in cases.items():
        g = device_block_gidx(ns, nd, s.contiguous(), d.contiguous())
        vin, w = g.position_operand(norm, "in")
        x = th.randn(ns, F, device=dev)
        out = th.empty(nd, F, device=dev)
        res[name + "_ms"] = ktime(lambda: K.binary_op_reduce("sum", "mul", vin, 0, 2, x, w, out))
        del g, vin, w, x, out
        th.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
