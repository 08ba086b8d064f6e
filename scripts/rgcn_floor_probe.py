#!/usr/bin/env python3
"""The gather floor under the fused R-GCN kernels on the C5 graph (Chung-Lu 5 M / 80 M,
4 relations, 64 -> 64, self-loop, bias): HIP-event medians of
  * copy_u_sum and u_mul_e_sum (the norm as edge weight) over the SAME graph with the
    headline load-balanced kernel -- the same 80 M random 256-B row gathers into the
    same destinations, with no relation split and no MFMA;
  * the fused layer-1 C entries (DGLMIRgcnLayer1Ex / BackwardEx on a prepared state),
    16-row kernel and (DGLMI_RGCN_TILE=32) the 32-row kernel.
So the fused forward can be read as a fraction of what a pure gather of its rows costs
on this box.  --prof: a few calls of each, for rocprofv3."""
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
    from bench_configs import chung_lu
    import dgl.function as fn
    from dgl import kernel as K
    dev = "cuda:0"
    n, m, R, f = 5_000_000, 80_000_000, 4, 64
    g = chung_lu(n, m, 0.5, 8, dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), generator=gen, device=dev)
    src, dst = g._graph._device_only
    indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
    norm = (1.0 / indeg)[dst.long()].reshape(m, 1).contiguous()
    x = th.randn(n, f, device=dev)
    gidx = g._graph.get_immutable_gidx(dev)
    steps = 3 if "--prof" in sys.argv else 10
    res = {"config": "C5 Chung-Lu 5M / 80M, 4 relations, 64 -> 64"}
    g.ndata["h"] = x
    g.edata["w"] = norm
    res["copy_u_sum_ms"] = ktime(lambda: g.update_all(fn.copy_u("h", "m"), fn.sum("m", "o")), steps)
    res["u_mul_e_sum_ms"] = ktime(lambda: g.update_all(fn.u_mul_e("h", "w", "m"), fn.sum("m", "o")),
                                  steps)
    from dgl import backend as B
    res["gcn_norm_aggregate_ms"] = ktime(lambda: B.gcn_norm_aggregate(gidx, x, "both"), steps)
    W = th.randn(R, f, f, device=dev) * 0.1
    Lw = th.randn(f, f, device=dev) * 0.1
    bias = th.randn(f, device=dev)
    et32 = et.int().contiguous()
    nf = norm.reshape(-1)
    K.rgcn_prepare(gidx, nf, R, layers=6, etypes=et32)
    ret = th.empty(n, f, device=dev)
    go = th.randn(n, f, device=dev)
    gh, gw, gl = th.empty(n, f, device=dev), th.empty_like(W), th.empty_like(Lw)
    for tile in ("16", "32"):
        os.environ["DGLMI_RGCN_TILE"] = tile
        res["fused%s_fwd_ms" % tile] = ktime(
            lambda: K.rgcn_layer1_ex(gidx, x, W, nf, ret, loop_weight=Lw, bias=bias, etypes=et32),
            steps)
        res["fused%s_bwd_ms" % tile] = ktime(
            lambda: K.rgcn_layer1_backward_ex(gidx, x, W, nf, Lw, go, gh, gw, gl, etypes=et32), steps)
        res["fused%s_bwd_nogradh_ms" % tile] = ktime(
            lambda: K.rgcn_layer1_backward_ex(gidx, x, W, nf, Lw, go, None, gw, gl, etypes=et32),
            steps)
    os.environ.pop("DGLMI_RGCN_TILE")
    # gather bytes per edge: a 256-B row + column + weight (+ row id in the fused walk)
    res["gather_GB"] = m * (256 + 8) / 1e9
    res["fused16_fwd_vs_copy_u_sum"] = res["fused16_fwd_ms"] / res["copy_u_sum_ms"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
