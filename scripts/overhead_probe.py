#!/usr/bin/env python3
"""Host-side cost of one message-passing call on a launch-bound graph (C1 Cora
size): DGLGraph.update_all(copy_u, sum) vs dgl.backend.copy_reduce vs
dgl.kernel.copy_reduce (the ctypes call) vs the kernel alone (HIP events), plus a
cProfile of update_all.  Output: gpurun_out/overhead_probe.json and .prof.txt."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import torch as th  # noqa: E402

import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from dgl import backend as B  # noqa: E402
from dgl import kernel as K  # noqa: E402


def per_call_us(f, n=3000):
    for _ in range(50):
        f()
    th.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    th.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    dev = "cuda:0"
    g = th.Generator(device=dev)
    g.manual_seed(1)
    n, m = 2708, 10556
    src = th.randint(0, n, (m,), device=dev, generator=g, dtype=th.int32)
    dst = th.randint(0, n, (m,), device=dev, generator=g, dtype=th.int32)
    gr = dgl.DGLGraph.from_device_coo(src, dst, n)
    x = th.randn(n, 16, device=dev)
    gr.ndata["h"] = x
    gidx = gr._graph.get_immutable_gidx(dev)
    out = th.empty(n, 16, device=dev)
    res = {"graph": "Cora-size random graph, 2708 nodes, 10556 edges, F = 16"}
    res["update_all_us"] = per_call_us(lambda: gr.update_all(fn.copy_u("h", "m"), fn.sum("m", "s")))
    res["backend_copy_reduce_us"] = per_call_us(lambda: B.copy_reduce("sum", gidx, 0, x, n))
    res["kernel_copy_reduce_us"] = per_call_us(lambda: K.copy_reduce("sum", gidx, 0, x, out))
    e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3000):
        K.copy_reduce("sum", gidx, 0, x, out)
    e1.record()
    th.cuda.synchronize()
    res["gpu_us_per_call_back_to_back"] = e0.elapsed_time(e1) / 3000 * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2000):
        gr.update_all(fn.copy_u("h", "m"), fn.sum("m", "s"))
    th.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/overhead_probe.prof.txt", "w") as fh:
        fh.write(s.getvalue())
    with open("gpurun_out/overhead_probe.json", "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
