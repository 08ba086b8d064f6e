#!/usr/bin/env python3
"""C3-size GATConv composition (use_fused = False: u_add_v SDDMM, LeakyReLU,
edge_softmax, u_mul_e_sum), HIP-event medians of each stage and of the module's
forward / forward + backward, for rocprofv3 kernel statistics (where the composition's
time goes next to the fused kernel's)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def ktime(fn, steps=5):
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
    from dgl import function as fn
    from dgl.nn.pytorch import GATConv, edge_softmax
    dev = "cuda:0"
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.4, 3, dev)
    x = th.randn(n, 602, device=dev)
    gat = GATConv(602, 8, 8).to(dev)
    gat.use_fused = False
    res = {"config": "C3 232965 nodes / 114.6 M edges, GATConv 602 -> 8 x 8, composition"}
    if "--module-only" in sys.argv:  # only module forward + backward steps (kernel stats)
        gat.attn_drop.p = float(os.environ.get("GAT_ATTN_DROP", "0"))
        for _ in range(4):
            gat(g, x).sum().backward()
        th.cuda.synchronize()
        print(json.dumps(res), flush=True)
        return
    with th.no_grad():
        ft = gat.fc(x).view(-1, 8, 8)
        el = (ft * gat.attn_l).sum(-1, keepdim=True)
        er = (ft * gat.attn_r).sum(-1, keepdim=True)
        lg = g.local_var()
        lg.srcdata.update({"ft": ft, "el": el})
        lg.dstdata.update({"er": er})

        def sddmm():
            lg.apply_edges(fn.u_add_v("el", "er", "e"))
        res["u_add_v_ms"] = ktime(sddmm)
        e = lg.edata["e"]
        res["leaky_relu_ms"] = ktime(lambda: gat.leaky_relu(e))
        e = gat.leaky_relu(e)
        res["edge_softmax_ms"] = ktime(lambda: edge_softmax(lg, e))
        lg.edata["a"] = edge_softmax(lg, e)
        res["u_mul_e_sum_ms"] = ktime(lambda: lg.update_all(fn.u_mul_e("ft", "a", "m"), fn.sum("m", "ft2")))

        # the same stages on the in-CSR position view (what GATConv now runs)
        import dgl.backend as B
        from dgl.nn.pytorch.softmax import _apply as softmax_on
        view = g._graph.get_immutable_gidx(dev).position_view("in")
        nd, m_ = view.num_dst, view.number_of_edges()
        res["pos_u_add_v_ms"] = ktime(lambda: B.binary_reduce("none", "add", view, B.SRC, B.DST, el, er, m_))
        ep = gat.leaky_relu(B.binary_reduce("none", "add", view, B.SRC, B.DST, el, er, m_))
        res["pos_edge_softmax_ms"] = ktime(lambda: softmax_on(view, ep, nd))
        ap = softmax_on(view, ep, nd)
        res["pos_u_mul_e_sum_ms"] = ktime(lambda: B.binary_reduce("sum", "mul", view, B.SRC, B.EDGE, ft, ap, nd))

        def fwd():
            gat(g, x)
        res["module_fwd_ms"] = ktime(fwd)

    def fwd_bwd():
        gat(g, x).sum().backward()
    res["module_fwd_bwd_ms"] = ktime(fwd_bwd)
    # the same module with the composition in edge-id order throughout (the reference's)
    from dgl.nn.pytorch.conv import gatconv
    gatconv.POSITION_SPACE = False
    with th.no_grad():
        res["edge_id_order_module_fwd_ms"] = ktime(fwd)
    res["edge_id_order_module_fwd_bwd_ms"] = ktime(fwd_bwd)
    gatconv.POSITION_SPACE = True
    # attention dropout 0.6 in training (nn.Dropout's edge-id draws; position space since
    # round 5), then the same in edge-id order
    gat.attn_drop.p = 0.6
    res["drop0.6_module_fwd_bwd_ms"] = ktime(fwd_bwd)
    gatconv.POSITION_SPACE = False
    res["drop0.6_edge_id_order_module_fwd_bwd_ms"] = ktime(fwd_bwd)
    gatconv.POSITION_SPACE = True
    gat.attn_drop.p = 0.0
    if "--kernels" in sys.argv:  # a few module steps for rocprofv3 kernel statistics
        for _ in range(3):
            fwd_bwd()
        th.cuda.synchronize()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
