#!/usr/bin/env python3
"""A/B timing of the fused GAT kernels on the C3 Reddit-size graph (232,965
nodes, 114.6 M edges, 8 heads x 8): forward and backward through the public
kernel wrappers (automatic column blocks, and unblocked), HIP-event medians.
Run once per library build (DGL_LIBRARY_PATH selects one); --save writes the
outputs so two builds can be compared (--compare A B)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch as th  # noqa: E402


def ev_time(fn, steps=10):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def run(args):
    from dgl import kernel as K
    from bench_configs import chung_lu
    dev = "cuda:0"
    H, D = 8, 8
    if args.graph == "m1":  # the bench's M1 graph (RMAT scale 23, 100 M edges)
        import dgl
        from bench import build_workload
        n, _, src, dst, _ = build_workload(1, 0, th.device(dev))
        g = dgl.DGLGraph.from_device_coo(src, dst, n)
    else:
        n, m = 232965, 114615892
        g = chung_lu(n, m, 0.4, 3, dev)
    gidx = g._graph.get_immutable_gidx(dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(3)
    ft = th.randn(n, H, D, device=dev, generator=gen)
    el = th.randn(n, H, device=dev, generator=gen)
    er = th.randn(n, H, device=dev, generator=gen)
    go = th.randn(n, H, D, device=dev, generator=gen)
    out = th.empty(n, H, D, device=dev)
    mx, sm = th.empty(n, H, device=dev), th.empty(n, H, device=dev)
    gft, gel, ger = th.empty_like(ft), th.empty_like(el), th.empty_like(er)
    ind = gidx.in_csr.indices.long()
    ghash = int((ind * th.arange(1, ind.numel() + 1, device=dev) % 1000003).sum().item())
    res = {"lib": os.environ.get("DGL_LIBRARY_PATH", "in-tree"), "graph_hash": ghash,
           "col_blocks": K.gat_col_blocks(gidx, ft)}
    saved = {}
    for blocks in (os.environ.get("GAT_AB_BLOCKS", "auto 1")).split():
        if blocks != "auto":
            os.environ["DGLMI_GAT_BLOCKS"] = blocks
        # GAT_AB_POS: the backward's edge-position path (1), destination-side walk (0), or
        # the forward's slope aggregates and no destination walk at all ("slopes")
        lf, ls = th.empty_like(out), th.empty_like(mx)
        for pos in (os.environ.get("GAT_AB_POS", "slopes 1")).split():
            os.environ["DGLMI_GAT_EDGE_POS"] = "1" if pos == "slopes" else pos
            key = blocks + {"slopes": "_slopes", "1": "", "0": "_dstwalk"}[pos]
            sl = (lf, ls) if pos == "slopes" else (None, None)
            fwd = lambda: K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm, *sl)
            bwd = lambda: K.fused_gat_backward(gidx, ft, el, er, 0.2, out, mx, sm, go, gft, gel, ger,
                                               *sl)
            res["fwd_ms_" + key] = ev_time(fwd)
            res["bwd_ms_" + key] = ev_time(bwd)
            fwd()
            bwd()
            th.cuda.synchronize()
            saved[key] = [t.cpu().clone() for t in (out, mx, sm, gft, gel, ger)]
            if key != blocks and blocks in saved:
                d = (saved[key][5].double() - saved[blocks][5].double()).abs()
                res["g_er_maxabs_%s_vs_pos" % key] = float(d.max())
                res["g_ft_equal_%s_vs_pos" % key] = bool(th.equal(saved[key][3], saved[blocks][3]))
    os.environ.pop("DGLMI_GAT_BLOCKS", None)
    os.environ.pop("DGLMI_GAT_EDGE_POS", None)
    if args.save:
        th.save(saved, args.save)
    print(json.dumps(res), flush=True)


def compare(a, b):
    A, B = th.load(a, weights_only=True), th.load(b, weights_only=True)
    res = {}
    for k in A:
        for name, x, y in zip(("out", "m", "l", "g_ft", "g_el", "g_er"), A[k], B[k]):
            d = (x.double() - y.double()).abs()
            res["%s_%s" % (k, name)] = {"max_abs": float(d.max()),
                                        "max_rel": float((d / y.double().abs().clamp(min=1e-3)).max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", default=None)
    ap.add_argument("--compare", nargs=2, default=None)
    ap.add_argument("--graph", default="c3", choices=["c3", "m1"])
    args = ap.parse_args()
    if args.compare:
        compare(*args.compare)
    else:
        run(args)
