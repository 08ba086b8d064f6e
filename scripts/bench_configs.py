#!/usr/bin/env python3
"""Secondary benchmarks for the BASELINE.json configs other than the headline:

  C1  2-layer GraphConv on a Cora-sized graph (2,708 nodes / 13,264 edges incl.
      self-loops, 1433 -> 16 -> 7): one training step (fwd + bwd + Adam)
  C2  GraphConv layer on an ogbn-arxiv-sized graph (169,343 / 1,166,243, F = 128)
  C3  GATConv (8 heads x 8) on a Reddit-sized graph (232,965 / 114,615,892,
      F_in = 602): forward + backward
  zoo the other conv modules (SAGE, GIN, SG, APPNP, TAG, Cheb, EdgeConv,
      GatedGraph) on the arxiv-size graph and SAGE-mean on the Reddit-size graph:
      forward + backward of the epilogue-fused form vs the reference-order form
  C5  RelGraphConv (4 relations, basis, 64 -> 64, per-edge norm) on 5,000,000
      nodes / 80,000,000 typed edges: forward + backward, and the typed gather alone

Graphs are synthetic Chung-Lu power-law graphs with the configs' (N, E) (the
datasets need network downloads).  Prints one JSON object per config.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

import dgl  # noqa: E402
from dgl.nn.pytorch import GraphConv, GATConv, FusedGATConv, RelGraphConv  # noqa: E402


def chung_lu(n, m, alpha, seed, device, self_loops=False):
    from dgl.data.synthetic import chung_lu_edges
    src, dst = chung_lu_edges(n, m, alpha, seed, device)  # the same draw on every rank
    if self_loops:
        ar = th.arange(n, device=device, dtype=th.int32)
        src = th.cat([src, ar])
        dst = th.cat([dst, ar])
    return dgl.DGLGraph.from_device_coo(src, dst, n)


def timeit(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    th.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    th.cuda.synchronize()
    return (time.perf_counter() - t) * 1000 / steps


def c1(dev, steps, warmup):
    g = chung_lu(2708, 10556, 0.5, 1, dev, self_loops=True)
    x = th.randn(2708, 1433, device=dev)
    y = th.randint(0, 7, (2708,), device=dev)
    l1, l2 = GraphConv(1433, 16, activation=th.relu).to(dev), GraphConv(16, 7).to(dev)
    params = list(l1.parameters()) + list(l2.parameters())
    opt = th.optim.Adam(params, lr=0.01, capturable=True)

    def step():
        opt.zero_grad(set_to_none=False)
        loss = th.nn.functional.cross_entropy(l2(g, l1(g, x)), y)
        loss.backward()
        opt.step()
    ms = timeit(step, steps, warmup)
    res = {"config": "C1 Cora-size 2-layer GCN train step", "nodes": 2708,
           "edges": g.number_of_edges(), "ms_per_step": ms}
    # the same step captured once into a HIP graph and replayed: the step is
    # ~40 small launches, so launch overhead, not the kernels, sets its time.
    # Fresh modules/optimizer (no autograd state from the eager runs), warm-up
    # on a side stream, then capture (torch.cuda.graphs whole-network recipe).
    try:
        m1, m2 = GraphConv(1433, 16, activation=th.relu).to(dev), GraphConv(16, 7).to(dev)
        ps = list(m1.parameters()) + list(m2.parameters())
        gopt = th.optim.Adam(ps, lr=0.01, capturable=True)

        def gstep():
            gopt.zero_grad(set_to_none=False)
            loss = th.nn.functional.cross_entropy(m2(g, m1(g, x)), y)
            loss.backward()
            gopt.step()
        s = th.cuda.Stream()
        s.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(s):
            for _ in range(3):
                gstep()
        th.cuda.current_stream().wait_stream(s)
        graph = th.cuda.CUDAGraph()
        with th.cuda.graph(graph):
            gstep()
        res["hipgraph_ms_per_step"] = timeit(graph.replay, steps * 10, warmup)
    except Exception as exc:  # report, keep the eager number
        res["hipgraph_error"] = repr(exc)[:300]
    return res


def c2(dev, steps, warmup):
    n, m, f = 169343, 1166243, 128
    g = chung_lu(n, m, 0.6, 2, dev)
    x = th.randn(n, f, device=dev, requires_grad=True)
    conv = GraphConv(f, f).to(dev)
    gidx = g._graph.get_immutable_gidx(dev)
    out = th.empty(n, f, device=dev)
    ms_spmm = timeit(lambda: dgl.kernel.copy_reduce("sum", gidx, 0, x.detach(), out), steps, warmup)

    def layer():
        x.grad = None  # as after zero_grad(set_to_none=True)
        conv.zero_grad(set_to_none=True)
        conv(g, x).sum().backward()
    ms = timeit(layer, steps, warmup)
    alg = 4 * (n + 1) + 4 * m + 4 * f * m + 4 * f * n
    res = {"config": "C2 arxiv-size GraphConv 128->128", "nodes": n, "edges": m,
           "copy_u_sum_ms": ms_spmm, "copy_u_sum_alg_GBps": alg / ms_spmm / 1e6,
           "copy_u_sum_Gedges_s": m / ms_spmm / 1e6, "layer_fwd_bwd_ms": ms}
    # the same layer step captured into a HIP graph: ~20 launches of 5-100 us each,
    # so the eager number carries the launch + Python overhead
    try:
        conv2 = GraphConv(f, f).to(dev)
        xg = th.randn(n, f, device=dev, requires_grad=True)

        def gstep():
            conv2(g, xg).sum().backward()
        st = th.cuda.Stream()
        st.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(st):
            for _ in range(3):
                gstep()
        th.cuda.current_stream().wait_stream(st)
        graph = th.cuda.CUDAGraph()
        with th.cuda.graph(graph):
            gstep()
        res["layer_fwd_bwd_hipgraph_ms"] = timeit(graph.replay, steps * 5, warmup)
    except Exception as exc:  # report, keep the eager number
        res["hipgraph_error"] = repr(exc)[:300]
    return res


def c3(dev, steps, warmup):
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.4, 3, dev)
    x = th.randn(n, 602, device=dev)
    gat = GATConv(602, 8, 8).to(dev)
    gat.use_fused = False  # the reference's unfused composition
    gat.train()

    def fwd():
        with th.no_grad():
            gat(g, x)

    def fwd_bwd():
        gat(g, x).sum().backward()
    ms_f = timeit(fwd, steps, warmup)
    ms_fb = timeit(fwd_bwd, steps, warmup)
    # the composition's step-by-step backward (round 5's) beside the fused one
    from dgl.nn.pytorch.conv import gatconv as _gatconv
    _gatconv.FUSED_COMPOSITION_BACKWARD = False
    ms_fb_step = timeit(fwd_bwd, steps, warmup)
    _gatconv.FUSED_COMPOSITION_BACKWARD = True
    fgat = FusedGATConv(602, 8, 8).to(dev)
    fgat.load_state_dict(gat.state_dict())

    def ffwd():
        with th.no_grad():
            fgat(g, x)

    def ffwd_bwd():
        fgat(g, x).sum().backward()
    ms_ff = timeit(ffwd, steps, warmup)
    ms_ffb = timeit(ffwd_bwd, steps, warmup)
    check = verify_gat_fused(gat, fgat, g, x)
    # training with the reference GAT example's attention dropout (train.py --attn-drop
    # 0.6): the composition applies nn.Dropout to the softmax; GATConv now keeps it in
    # the fused kernels
    dgat = GATConv(602, 8, 8, attn_drop=0.6).to(dev)
    dgat.load_state_dict(gat.state_dict())
    dgat.train()

    def dfwd_bwd():
        dgat(g, x).sum().backward()
    from dgl.nn.pytorch.conv import gatconv as gatconv_mod
    # the module's nn.Dropout draws (default: recomputed inside the walks when
    # dgl.kernel.dropout_draw_ok; the route actually taken is recorded)
    ms_dfb = timeit(dfwd_bwd, steps, warmup)
    from dgl import kernel as K
    draw_route = bool(gatconv_mod.MODULE_DRAW_IN_KERNEL and K.dropout_draw_ok(dev))
    gatconv_mod.MODULE_DRAW_IN_KERNEL = False
    ms_dfb_mask = timeit(dfwd_bwd, steps, warmup)  # torch's mask packed to keep words
    gatconv_mod.MODULE_DRAW_IN_KERNEL = True
    dgat.attn_drop_mask = "hashed"
    ms_dfb_hashed = timeit(dfwd_bwd, steps, warmup)  # opt-in hashed mask
    dgat.attn_drop_mask = "module"
    dgat.use_fused = False
    ms_dufb = timeit(dfwd_bwd, steps, warmup)
    return {"config": "C3 Reddit-size GATConv 602 -> 8x8", "nodes": n, "edges": m,
            "unfused_fwd_ms": ms_f, "unfused_fwd_bwd_ms": ms_fb,
            "unfused_stepwise_bwd_fwd_bwd_ms": ms_fb_step,
            "fused_fwd_ms": ms_ff, "fused_fwd_bwd_ms": ms_ffb,
            "fused_fwd_Gedges_s": m / ms_ff / 1e6, "fused_fwd_bwd_Gedges_s": m / ms_ffb / 1e6,
            "attn_drop_0.6_fused_fwd_bwd_ms": ms_dfb,
            "attn_drop_0.6_fused_draws_in_kernel": draw_route,
            "attn_drop_0.6_fused_torch_mask_fwd_bwd_ms": ms_dfb_mask,
            "attn_drop_0.6_fused_hashed_mask_fwd_bwd_ms": ms_dfb_hashed,
            "attn_drop_0.6_unfused_fwd_bwd_ms": ms_dufb,
            "check": check}


def verify_gat_fused(gat, fgat, g, x):
    """The fused kernels (FusedGATConv) against the unfused composition (GATConv with
    use_fused = False, same weights) on the timed C3 graph: output, input gradient and
    every parameter gradient under one random output gradient.  Raises on a mismatch."""
    xr = x.detach().clone().requires_grad_()
    go = th.randn(x.shape[0], 8, 8, device=x.device)
    res = []
    for mod in (gat, fgat):
        mod.zero_grad()
        xr.grad = None
        out = mod(g, xr)
        out.backward(go)
        res.append([out.detach(), xr.grad.clone()] + [p.grad.clone() for p in mod.parameters()])
    worst = 0.0
    for a, b in zip(*res):
        err = float((a - b).abs().max())
        bound = 1e-4 + 1e-4 * float(b.abs().max())
        worst = max(worst, err / bound)
        if err > bound:
            raise AssertionError("C3: fused differs from the composition by %.3g (bound %.3g)"
                                 % (err, bound))
    return {"fused_vs_unfused_checked": True, "worst_err_over_bound": worst,
            "compared": "output, x.grad and parameter grads; bound 1e-4 + 1e-4 max|composition|"}


def verify_rgcn_fused(conv, g, x, et, norm):
    """The fused R-GCN route vs the GEMM + typed-gather route, once, before any C5
    time is taken: output (rtol = atol = 1e-4) and the input and every parameter
    gradient (|a - b| <= 1e-3 + 1e-4 max|b|: long fp32 sums in two orders).  Raises,
    so a wrong fast kernel cannot print a time."""
    gen = th.Generator(device=x.device)
    gen.manual_seed(11)
    params = [x] + list(conv.parameters())
    res = {}
    for fused in (True, False):
        conv.use_fused = fused
        out = conv(g, x, et, norm)
        if fused and g._graph.__dict__.get("_rgcn_fused") is None:
            raise AssertionError("C5: the fused route did not run")
        go = th.randn(out.shape, device=x.device, generator=gen) if fused else go
        res[fused] = (out.detach(), th.autograd.grad(out, params, go))
        del out
    conv.use_fused = True
    (fo, fg), (uo, ug) = res[True], res[False]
    if not th.allclose(fo, uo, rtol=1e-4, atol=1e-4):
        raise AssertionError("C5: fused output differs from the unfused route by %.3g"
                             % float((fo - uo).abs().max()))
    worst = 0.0
    for a, b in zip(fg, ug):
        bound = 1e-3 + 1e-4 * float(b.abs().max())
        err = float((a - b).abs().max())
        worst = max(worst, err / bound)
        if err > bound:
            raise AssertionError("C5: fused gradient differs by %.3g (bound %.3g)" % (err, bound))
    return {"fused_vs_unfused_checked": True, "out_max_abs_diff": float((fo - uo).abs().max()),
            "grad_worst_err_over_bound": worst}


def c5(dev, steps, warmup):
    n, m, R, f = 5_000_000, 80_000_000, 4, 64
    g = chung_lu(n, m, 0.5, 8, dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), generator=gen, device=dev)
    src, dst = g._graph._device_only
    indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
    norm = (1.0 / indeg)[dst.long()].reshape(m, 1)
    x = th.randn(n, f, device=dev, requires_grad=True)
    conv = RelGraphConv(f, f, R, "basis", num_bases=R, self_loop=True).to(dev)
    check = verify_rgcn_fused(conv, g, x, et, norm)

    def fwd_bwd():
        # gradients start from None each step, as after an optimizer's
        # zero_grad(set_to_none=True): no accumulation pass over x.grad (5 M x 64)
        x.grad = None
        conv.zero_grad(set_to_none=True)
        conv(g, x, et, norm).sum().backward()

    def fwd():
        with th.no_grad():
            conv(g, x, et, norm)
    ms_fb = timeit(fwd_bwd, steps, warmup)
    ms_f = timeit(fwd, steps, warmup)
    fused = g._graph.__dict__.get("_rgcn_fused") is not None
    conv.use_fused = False  # the GEMM + typed-gather path, for comparison
    ms_fb_u = timeit(fwd_bwd, steps, warmup)
    ms_f_u = timeit(fwd, steps, warmup)
    conv.use_fused = True
    from dgl import backend as B
    y = th.randn(R * n, f, device=dev)
    ms_g = timeit(lambda: B._typed_aggregate(g, R, y, norm, et), steps, warmup)
    # typed gather (u_mul_e_sum, edge weight broadcast): idx + eid + row + weight per
    # edge, indptr + output row per node
    alg = 4 * (n + 1) + m * (4 + 4 + 4 * f + 4) + 4 * f * n
    return {"config": "C5 R-GCN RelGraphConv 4 rel basis 64->64", "nodes": n, "edges": m,
            "layer_fwd_ms": ms_f, "layer_fwd_bwd_ms": ms_fb, "fused_route": fused,
            "gemm_gather_fwd_ms": ms_f_u, "gemm_gather_fwd_bwd_ms": ms_fb_u,
            "typed_gather_ms": ms_g,
            "typed_gather_alg_GBps": alg / ms_g / 1e6, "typed_gather_Gedges_s": m / ms_g / 1e6,
            "check": check}


def sd(dev, steps, warmup):
    """g-SDDMM on the M1 graph (RMAT scale 23, 100M edges): u_dot_v with F = 64
    (link-prediction scoring) and u_add_v with H = 8 (GAT logits), in both item
    orders.  Algorithmic bytes per edge: u_dot_v 8 + 8F + 4;
    u_add_v 8 + 2*4H + 4H."""
    import bench
    n, n_dst, src, dst, x = bench.build_workload(1, 0, dev)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    gidx = g._graph.get_immutable_gidx(dev)
    m = int(src.shape[0])
    del src, dst
    el = th.rand(n, 8, device=dev)
    er = th.rand(n, 8, device=dev)
    res = {"config": "SDDMM on M1 (RMAT scale 23, 100M edges)", "nodes": n, "edges": m}
    cases = [("u_dot_v_F64", "dot", x, x, 8 + 8 * 64 + 4),
             ("u_add_v_H8", "add", el, er, 8 + 2 * 32 + 32)]
    for name, op, a, b, per_edge in cases:
        for order in ("auto", "coo", "csr"):
            dgl.kernel.set_sddmm_order(order)
            try:
                ms = timeit(lambda: dgl.backend.binary_reduce("none", op, gidx, 0, 1, a, b, m),
                            steps, warmup)
            finally:
                dgl.kernel.set_sddmm_order("auto")
            res["%s_%s_ms" % (name, order)] = ms
            res["%s_%s_alg_GBps" % (name, order)] = per_edge * m / ms / 1e6
    return res


def c5h(dev, steps, warmup):
    """C5 as a heterograph: 4 relations node -> node (20 M edges each), copy_u +
    sum per relation, cross-type sum -- multi_update_all's fused path (one SpMM
    over the merged relations) against one SpMM per relation + torch sum."""
    n, m, R, f = 5_000_000, 80_000_000, 4, 64
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    rels = {}
    for r in range(R):
        src = th.randint(0, n, (m // R,), generator=gen, device=dev)
        dst = th.randint(0, n, (m // R,), generator=gen, device=dev)
        rels[("node", "r%d" % r, "node")] = (src, dst)
    g = dgl.heterograph(rels, {"node": n})
    g.nodes["node"].data["h"] = th.randn(n, f, device=dev)
    funcs = {"r%d" % r: (dgl.function.copy_src("h", "m"), dgl.function.sum("m", "o"))
             for r in range(R)}
    ms_fused = timeit(lambda: g.multi_update_all(funcs, "sum"), steps, warmup)
    ms_loop = timeit(lambda: g.multi_update_all(funcs, "max"), steps, warmup)

    def per_rel_sum():
        outs = []
        for r in range(R):
            rel = g["r%d" % r].local_var()
            rel.update_all(dgl.function.copy_src("h", "m"), dgl.function.sum("m", "o"))
            outs.append(rel.dstdata["o"])
        return sum(outs)
    ms_unfused = timeit(per_rel_sum, steps, warmup)
    return {"config": "C5 heterograph 4 relations, multi_update_all copy_u/sum", "nodes": n,
            "edges": m, "fused_cross_sum_ms": ms_fused, "per_relation_then_sum_ms": ms_unfused,
            "per_relation_cross_max_ms": ms_loop,
            "fused_Gedges_s": m / ms_fused / 1e6}


def gemm(dev, steps, warmup):
    """The dense feature projections that bracket the aggregations (MFMA via
    hipBLASLt, fp32 in / fp32 accumulate like the reference): forward X W and the
    two backward GEMMs, at each config's shape.  Utilisation = achieved TFLOP/s /
    157.3 TFLOP/s (MI355X dense FP32 matrix peak, MI355X_MICROARCH.md)."""
    peak = 157.3
    shapes = {"C1 layer1 2708x1433->16": (2708, 1433, 16),
              "C2 169343x128->128": (169343, 128, 128),
              "C3 GAT fc 232965x602->64": (232965, 602, 64),
              "C5 R-GCN 5Mx64->4x64": (5_000_000, 64, 256)}
    res = {"config": "bracketing GEMMs (fp32, torch.matmul -> hipBLASLt MFMA)"}
    for name, (m, k, n) in shapes.items():
        x = th.randn(m, k, device=dev)
        w = th.randn(k, n, device=dev)
        gy = th.randn(m, n, device=dev)
        fl = 2.0 * m * k * n
        for tag, fn in (("fwd", lambda: x @ w), ("grad_x", lambda: gy @ w.t()),
                        ("grad_w", lambda: x.t() @ gy)):
            ms = timeit(fn, steps, warmup)
            res["%s %s ms" % (name, tag)] = ms
            res["%s %s TFLOPs" % (name, tag)] = fl / ms / 1e9
            res["%s %s mfma_util" % (name, tag)] = fl / ms / 1e9 / peak
    return res


def zoo(dev, steps, warmup):
    import dgl.nn.pytorch as nn
    res = {"config": "conv module zoo, fwd+bwd ms: fused / reference order"}
    n, m, f = 169343, 1166243, 128
    g = chung_lu(n, m, 0.6, 2, dev)
    etypes = th.randint(0, 4, (m,), device=dev)
    mods = {
        "SAGE_mean_128_128": (nn.SAGEConv(f, f, "mean"), ()),
        "SAGE_gcn_128_128": (nn.SAGEConv(f, f, "gcn"), ()),
        "GIN_sum_128": (nn.GINConv(th.nn.Linear(f, f), "sum"), ()),
        "GIN_mean_128": (nn.GINConv(th.nn.Linear(f, f), "mean"), ()),
        "SGConv_k2_128_64": (nn.SGConv(f, 64, k=2), ()),
        "APPNP_k10_128": (nn.APPNPConv(10, 0.1), ()),
        "TAGConv_k2_128_64": (nn.TAGConv(f, 64, k=2), ()),
        "ChebConv_k3_128_64": (nn.ChebConv(f, 64, 3), ([2.0],)),
        "EdgeConv_128_64": (nn.EdgeConv(f, 64), ()),
        "GatedGraph_4types_128_1step": (nn.GatedGraphConv(f, f, 1, 4), (etypes,)),
    }
    x = th.randn(n, f, device=dev, requires_grad=True)
    for name, (mod, extra) in mods.items():
        mod = mod.to(dev)
        for fused in (True, False):
            mod.fused = fused

            def step():
                mod(g, x, *extra).sum().backward()
            res["%s_%s" % (name, "fused" if fused else "ref")] = timeit(step, steps, warmup)
        res[name + "_speedup"] = res[name + "_ref"] / res[name + "_fused"]
    del g, x
    th.cuda.empty_cache()
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.6, 3, dev)
    x = th.randn(n, 602, device=dev, requires_grad=True)
    mod = nn.SAGEConv(602, 64, "mean").to(dev)
    for fused in (True, False):
        mod.fused = fused

        def step():
            mod(g, x).sum().backward()
        res["Reddit_SAGE_mean_602_64_%s" % ("fused" if fused else "ref")] = \
            timeit(step, max(2, steps // 2), 1)
    res["Reddit_SAGE_mean_602_64_speedup"] = (res["Reddit_SAGE_mean_602_64_ref"]
                                              / res["Reddit_SAGE_mean_602_64_fused"])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3,c5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    dev = "cuda:0"
    for c in args.configs.split(","):
        res = globals()[c](dev, args.steps, args.warmup)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
