#!/usr/bin/env python3
"""The load-balanced reduce's edge-value kinds on one graph (the C5 Chung-Lu graph,
5 M nodes / 80 M edges, F = 64): HIP-event medians of copy_u_sum (the floor: one
256-B row per edge), u_mul_e_sum with a constant weight (streamed in walk order from
its second use), u_mul_e_sum with a fresh broadcast operand per call ((N, 8, 8) x
(E, 8, 1), the unfused GAT aggregation), copy_u_max forward and its source gradient
(the tie mask: two gathered rows per edge).  --graph m1: the headline RMAT graph."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def ktime(fn, steps=10):
    fn()
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    import dgl
    import dgl.function as fn
    from bench_configs import chung_lu
    dev = "cuda:0"
    if "m1" in sys.argv:
        import bench
        n, _, src, dst, x = bench.build_workload(1, 0, dev)
        g = dgl.DGLGraph.from_device_coo(src, dst, n)
        del src, dst
        m = g.number_of_edges()
    elif "sorted" in sys.argv:
        # the C5 graph with its edges in destination order: edge ids = in-CSR positions
        # (DGLMIGraph.eid_identity); DGLMI_EID_IDENTITY=0 in the environment for the A/B
        from dgl.data.synthetic import chung_lu_edges
        n, m = 5_000_000, 80_000_000
        src, dst = chung_lu_edges(n, m, 0.5, 8, dev)
        order = th.sort(dst.long() * n + src.long()).indices  # (destination, source) order
        g = dgl.DGLGraph.from_device_coo(src[order].contiguous(), dst[order].contiguous(), n)
        del src, dst, order
        x = th.randn(n, 64, device=dev)
    else:
        n, m = 5_000_000, 80_000_000
        g = chung_lu(n, m, 0.5, 8, dev)
        x = th.randn(n, 64, device=dev)
    res = {"graph": "m1" if "m1" in sys.argv else ("c5 chung-lu, dst-sorted edge ids" if "sorted" in sys.argv
                                                    else "c5 chung-lu"), "nodes": n, "edges": m,
           "eid_identity": g._graph.get_immutable_gidx(dev).eid_identity_bits()}
    g.ndata["x"] = x
    g.edata["w"] = th.rand(m, 1, device=dev)
    res["copy_u_sum_ms"] = ktime(lambda: g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")))
    res["u_mul_e_sum_const_w_ms"] = ktime(lambda: g.update_all(fn.u_mul_e("x", "w", "m"),
                                                               fn.sum("m", "o")))
    xh = x.view(n, 8, 8)
    g.ndata["xh"] = xh

    def fresh_bcast():
        g.edata["a"] = th.rand(m, 8, 1, device=dev)  # a new tensor per call
        g.update_all(fn.u_mul_e("xh", "a", "m"), fn.sum("m", "oh"))
    a0 = th.rand(m, 8, 1, device=dev)
    res["alloc_only_ms"] = ktime(lambda: th.rand(m, 8, 1, device=dev))
    res["u_mul_e_sum_bcast_fresh_ms_incl_alloc"] = ktime(fresh_bcast)
    del a0
    res["copy_u_max_ms"] = ktime(lambda: g.update_all(fn.copy_u("x", "m"), fn.max("m", "o")))
    xr = x.clone().requires_grad_()
    g.ndata["xr"] = xr
    g.update_all(fn.copy_u("xr", "m"), fn.max("m", "omax"))
    out = g.ndata["omax"]
    go = th.randn_like(out)
    res["copy_u_max_backward_ms"] = ktime(
        lambda: th.autograd.grad(out, (xr,), go, retain_graph=True))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
