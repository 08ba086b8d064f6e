#!/usr/bin/env python3
"""u_mul_e_sum with a per-head attention (the GAT composition's aggregation, C3 size) on
the in-CSR position view: forward (in-CSR walk, attention streamed) and the node gradient
(out-CSR walk, attention read at random positions) under the probe build's kernel
variants (DGLMI_PROBES=1, DGLMI_SPMM_VARIANT: 3 shipped, 0 plain loads, 1 non-temporal
CSR loads only, 7 twice the gathers in flight).  HIP-event medians; outputs compared with
the shipped variant's."""
import json
import os
import sys

os.environ["DGLMI_PROBES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def ktime(fn, steps=7):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    from bench_configs import chung_lu
    import dgl.backend as B
    from dgl import kernel as K
    dev = "cuda:0"
    g = chung_lu(232965, 114615892, 0.4, 3, dev)
    view = g._graph.get_immutable_gidx(dev).position_view("in")
    nd, m = view.num_dst, view.number_of_edges()
    gen = th.Generator(device=dev).manual_seed(5)
    ft = th.randn(nd, 8, 8, device=dev, generator=gen)
    a = th.rand(m, 8, 1, device=dev, generator=gen)
    grad = th.randn(nd, 8, 8, device=dev, generator=gen)
    out = th.empty(nd, 8, 8, device=dev)
    gn = th.empty_like(ft)
    res, ref = {}, None
    for var in ("3", "0", "1", "7"):
        os.environ["DGLMI_SPMM_VARIANT"] = var
        fwd = lambda: K.binary_op_reduce("sum", "mul", view, B.SRC, B.EDGE, ft, a, out)  # noqa: E731
        bwd = lambda: K.backward_lhs_binary_op_reduce("sum", "mul", view, B.SRC, B.EDGE, ft, a,  # noqa: E731
                                                      out, grad, gn)
        res["var%s_fwd_ms" % var] = ktime(fwd)
        res["var%s_node_grad_ms" % var] = ktime(bwd)
        fwd()
        bwd()
        th.cuda.synchronize()
        if ref is None:
            ref = (out.clone(), gn.clone())
        else:
            res["var%s_bit_identical" % var] = bool(th.equal(out, ref[0]) and th.equal(gn, ref[1]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
