#!/usr/bin/env python3
"""Experiment: column blocks for the load-balanced copy_u_sum on a high-degree
graph whose feature table fits the Infinity Cache but not L2 (Reddit-size,
232,965 nodes, 114.6 M edges, F = 64 -> 60 MB).  Sums the per-source-block
launch times (no merge) against the whole-graph launch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

from dgl import kernel as K  # noqa: E402
from dgl.graph_index import device_block_gidx  # noqa: E402
from bench_configs import chung_lu  # noqa: E402


def ktime(fn, steps=6):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    dev = "cuda:0"
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.4, 3, dev)
    src, dst = (t.to(dev) for t in g._graph._device_only)
    gidx = g._graph.get_immutable_gidx(th.device(dev))
    res = {}
    for f in (64, 128):
        x = th.randn(n, f, device=dev)
        out = th.empty(n, f, device=dev)
        res["F%d_whole_ms" % f] = ktime(lambda: K.copy_reduce("sum", gidx, 0, x, out))
        for nb in (4, 8, 16):
            bounds = [n * b // nb for b in range(nb + 1)]
            tot = 0.0
            for b in range(nb):
                sel = (src >= bounds[b]) & (src < bounds[b + 1])
                sg = device_block_gidx(n, n, src[sel], dst[sel])
                tot += ktime(lambda: K.copy_reduce("sum", sg, 0, x, out))
                del sg
            res["F%d_blocks%d_sum_ms" % (f, nb)] = tot
    # the shipped path: chained passes over the cached blocks (DGLMI_SPMM_BLOCKS)
    m_e = gidx.in_csr.nnz
    for f in (64, 128):
        x = th.randn(n, f, device=dev)
        out = th.empty(n, f, device=dev)
        a = th.rand(m_e, 8, 1, device=dev)
        for nb in ("1", "8", "16"):
            os.environ["DGLMI_SPMM_BLOCKS"] = nb
            res["F%d_copy_u_sum_blocks%s_ms" % (f, nb)] = ktime(
                lambda: K.copy_reduce("sum", gidx, 0, x, out))
            res["F%d_u_mul_e_bcast_blocks%s_ms" % (f, nb)] = ktime(
                lambda: K.binary_op_reduce("sum", "mul", gidx, "src", "edge", x.view(n, 8, f // 8),
                                           a, out.view(n, 8, f // 8)))
        os.environ.pop("DGLMI_SPMM_BLOCKS")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
