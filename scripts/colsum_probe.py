#!/usr/bin/env python3
"""Reductions over the leading dim that bracket the projections: the split-K
weight gradient's slice sum (S x k x n -> k x n) and bias gradients (N x F -> F).
Torch's sum(0) on a short leading dim took 0.5 ms in the C2 trace; this times it
against a GEMV (ones @ view) and a two-level sum."""
import json
import time

import torch as th

dev = "cuda:0"


def t(fn, n=50):
    fn()
    th.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(n):
        fn()
    th.cuda.synchronize()
    return (time.perf_counter() - s) * 1e3 / n


res = {}
for S, k, n in ((128, 128, 128), (128, 64, 256), (64, 602, 64), (128, 16, 1433)):
    p = th.randn(S, k, n, device=dev)
    ones = th.ones(1, S, device=dev)
    key = "%dx%dx%d" % (S, k, n)
    res[key + " sum0"] = t(lambda: p.sum(0))
    res[key + " ones_mm"] = t(lambda: (ones @ p.view(S, k * n)).view(k, n))
    res[key + " view_sum0"] = t(lambda: p.view(S, k * n).sum(0))
    ref = p.double().sum(0)
    res[key + " ones_mm_err"] = float(((ones @ p.view(S, k * n)).view(k, n).double() - ref).abs().max())
for N, F in ((169343, 128), (232965, 64), (5000000, 64)):
    g = th.randn(N, F, device=dev)
    res["%dx%d sum0" % (N, F)] = t(lambda: g.sum(0))
print(json.dumps(res, indent=0))
