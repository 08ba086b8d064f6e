#!/usr/bin/env python3
"""C5 typed gather (R-GCN aggregation over the relation-expanded graph, 5 M nodes,
80 M edges, 4 relations, F = 64): where its time goes.  Times the gather with the
per-edge norm (u_mul_e sum, the shipped path), without it (copy_u sum, which also
gets the cold-row hints), and with the norm pre-permuted into in-CSR position
order (edge operand streamed instead of gathered by edge id)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

from dgl import backend as B  # noqa: E402
from dgl import kernel as K  # noqa: E402
from dgl.graph_index import DeviceCSR, ImmutableGraphIndex  # noqa: E402
from bench_configs import chung_lu  # noqa: E402


def ktime(fn, steps=10):
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
    n, m, R, f = 5_000_000, 80_000_000, 4, 64
    g = chung_lu(n, m, 0.5, 8, dev)
    gen = th.Generator(device=dev)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), generator=gen, device=dev)
    src, dst = g._graph._device_only
    indeg = th.bincount(dst.long(), minlength=n).float().clamp(min=1)
    norm = (1.0 / indeg)[dst.long()].reshape(m, 1)
    y = th.randn(n * R, f, device=dev)
    tg = g._graph.typed_gidx(th.device(dev), R, et, True)
    out = th.empty(n, f, device=dev)
    res = {}
    res["u_mul_e_ms"] = ktime(lambda: B._typed_aggregate(g, R, y, norm, et, node_major=True))
    res["copy_u_ms"] = ktime(lambda: K.copy_reduce("sum", tg, 0, y, out))
    os.environ["DGLMI_HOT_DEGREE"] = "0"
    tg._gather_cols = None
    res["copy_u_nohints_ms"] = ktime(lambda: K.copy_reduce("sum", tg, 0, y, out))
    os.environ.pop("DGLMI_HOT_DEGREE")
    tg._gather_cols = None
    # position-ordered edge operand: a view of the typed graph whose edge ids are
    # the in-CSR positions
    ic, oc = tg.in_csr, tg.out_csr
    pos = th.arange(ic.nnz, device=dev, dtype=th.int32)
    inv = th.empty_like(pos)
    inv[ic.data.long()] = pos
    pv = ImmutableGraphIndex(DeviceCSR(ic.indptr, ic.indices, pos, ic.rows, ic.num_cols),
                             DeviceCSR(oc.indptr, oc.indices, inv[oc.data.long()], oc.rows, oc.num_cols),
                             tg.num_src, tg.num_dst, tg.device, eid_perm=True)
    npos = norm[ic.data.long()].contiguous()
    res["u_mul_e_posorder_ms"] = ktime(
        lambda: K.binary_op_reduce("sum", "mul", pv, "src", "edge", y, npos, out))
    ref = th.empty_like(out)
    K.binary_op_reduce("sum", "mul", tg, "src", "edge", y, norm, ref)
    res["posorder_max_abs_diff"] = float((out - ref).abs().max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
