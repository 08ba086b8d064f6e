#!/usr/bin/env python3
"""Would splitting the feature dimension help the headline copy_u_sum?  On the M1
graph, time copy_u_sum over the full F = 64 table against passes over narrower
column slices stored as their own tables (F = 32 x 2, F = 16 x 4): a narrower
table keeps a larger share of its rows in the Infinity Cache."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import torch as th  # noqa: E402

import bench  # noqa: E402
from dgl import kernel as K  # noqa: E402

dev = "cuda:0"
th.cuda.set_device(0)
n, n_dst, src, dst, x = bench.build_workload(1, 0, dev)
gidx, _ = bench.make_local_graph(n, n_dst, src, dst, dev)
del src, dst


def t(fn, reps=10):
    for _ in range(3):
        fn()
    s, e = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    th.cuda.synchronize()
    return s.elapsed_time(e) / reps


res = {}
out = th.empty(n_dst, 64, device=dev)
res["F64_ms"] = t(lambda: K.copy_reduce("sum", gidx, 0, x, out))
for w in (32, 16):
    parts = [x[:, i:i + w].contiguous() for i in range(0, 64, w)]
    outs = [th.empty(n_dst, w, device=dev) for _ in parts]

    def run():
        for p, o in zip(parts, outs):
            K.copy_reduce("sum", gidx, 0, p, o)
    res["F%dx%d_ms" % (w, 64 // w)] = t(run)
    del parts, outs
print(json.dumps(res))
