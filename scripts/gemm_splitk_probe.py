#!/usr/bin/env python3
"""Probe: weight-gradient GEMMs dW = X^T dY with a huge reduction dim (N nodes)."""
import json
import time
import torch as th


def timeit(fn, steps=10, warmup=3):
    for _ in range(warmup):
        fn()
    th.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    th.cuda.synchronize()
    return (time.perf_counter() - t) * 1000 / steps


dev = "cuda:0"
res = {}
for m, k, n in [(169343, 128, 128), (232965, 602, 64), (5_000_000, 64, 256), (5_000_000, 64, 64)]:
    x = th.randn(m, k, device=dev)
    gy = th.randn(m, n, device=dev)
    ref = x.t() @ gy
    key = "%dx%dx%d" % (m, k, n)
    res[key + " xt@gy"] = timeit(lambda: x.t() @ gy)
    res[key + " (gyt@x)t"] = timeit(lambda: (gy.t() @ x).t())
    for S in (8, 32, 128, 512):
        mm = (m // S) * S
        def f():
            a = th.bmm(x[:mm].view(S, mm // S, k).transpose(1, 2), gy[:mm].view(S, mm // S, n)).sum(0)
            if mm < m:
                a += x[mm:].t() @ gy[mm:]
            return a
        err = float((f() - ref).abs().max() / ref.abs().max())
        res[key + " bmm S=%d" % S] = timeit(f)
        res[key + " bmm S=%d relerr" % S] = err
    res[key + " addmm chunks"] = None
print(json.dumps(res, indent=1))
