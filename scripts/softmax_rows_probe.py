#!/usr/bin/env python3
"""Fused edge softmax on the C3 graph (232,965 nodes / 114.6 M edges), H = 8 and
H = 1 (--quad: H = 1, 2 and 4 on the view and the graph, four values per lane against one): forward and backward HIP-event medians on the graph, on its in-CSR position
view with the chunked row + edge passes, and on the view with the row-owned walk, plus a digest of every output (run against two builds of the library to
show bit-identity)."""
import hashlib
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
    from dgl import kernel as K
    dev = "cuda:0"
    g = chung_lu(232965, 114615892, 0.4, 3, dev)
    gidx = g._graph.get_immutable_gidx(dev)
    res = {"lib": os.environ.get("DGL_LIBRARY_PATH", "in-tree")}
    dig = hashlib.sha256()
    # --pmc: H = 8 (or with --pmc-h1 H = 1) on the view only (chunked, then row-owned),
    # for counter passes
    pmc = "--pmc" in sys.argv
    pmc_h = 1 if "--pmc-h1" in sys.argv else 8  # --pmc --pmc-h1: the H = 1 view instead
    quad_only = "--quad" in sys.argv  # H = 1 / 2 on the view: four values per lane vs one
    hs = (1, 2, 4) if quad_only else ((pmc_h,) if pmc else ((1, 2, 4, 8, 16) if "--pack" in sys.argv else (8, 1)))
    for H in hs:
        gen = th.Generator(device=dev).manual_seed(H)
        s = th.randn(gidx.number_of_edges(), H, 1, device=dev, generator=gen) * 3
        ga = th.randn(s.shape, device=dev, generator=gen)
        view = gidx.position_view("in")
        routes = (("graph", gidx, "1", "1"), ("view_chunked", view, "0", "1"), ("view", view, "1", "1"))
        if quad_only:
            routes = (("view_plain", view, "1", "0"), ("view", view, "1", "1"),
                      ("graph_plain", gidx, "1", "0"), ("graph", gidx, "1", "1"))
        elif "--pack" in sys.argv:  # the edge-id route with / without packed row statistics
            routes = (("graph_unpacked", gidx, "1", "1", "0"), ("graph", gidx, "1", "1", "1"))
        elif pmc:
            routes = routes[1:]
        for name, gi, owned, quad, *pack in routes:
            os.environ["DGLMI_SOFTMAX_OWNED"] = owned  # 0: the chunked row + edge passes
            os.environ["DGLMI_SOFTMAX_QUAD"] = quad  # 0: one position per lane at H <= 4
            os.environ["DGLMI_SOFTMAX_PACK"] = pack[0] if pack else "1"  # 0: two statistics arrays
            out, gs = th.empty_like(s), th.empty_like(s)
            res["H%d_%s_fwd_ms" % (H, name)] = ktime(lambda: K.edge_softmax_forward(gi, s, out))
            res["H%d_%s_bwd_ms" % (H, name)] = ktime(lambda: K.edge_softmax_backward(gi, out, ga, gs))
            for t in (out, gs):
                dig.update(t.cpu().numpy().tobytes())
            # operand bytes: forward reads the logits and writes the softmax, backward
            # reads the softmax and its gradient and writes the logits' gradient
            nb = s.numel() * 4
            res["H%d_%s_fwd_TBps" % (H, name)] = 2 * nb / res["H%d_%s_fwd_ms" % (H, name)] / 1e9
            res["H%d_%s_bwd_TBps" % (H, name)] = 3 * nb / res["H%d_%s_bwd_ms" % (H, name)] / 1e9
    res["digest"] = dig.hexdigest()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
