#!/usr/bin/env python3
"""Tuning sweep of the fused GAT kernels on the C3 Reddit-size graph: chunk size
(DGLMI_CHUNK_EDGES) x gathers in flight per lane (DGLMI_GAT_U, read by a build
with the U template variants -- removed after the sweep in
profiles/r01_tune_gat.json showed the shipped U = 8 best; the release build
ignores it), kernel-level forward and backward times with HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

# the policy / tuning variants live in the probe build (make -C dgl-hack_amd PROBES=1)
os.environ.setdefault("DGLMI_PROBES", "1")

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

from dgl import kernel as K  # noqa: E402
from bench_configs import chung_lu  # noqa: E402


def ev_time(fn, steps=8):
    fn()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    th.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


dev = "cuda:0"
n, m, H, D = 232965, 114615892, 8, 8
g = chung_lu(n, m, 0.4, 3, dev)
gidx = g._graph.get_immutable_gidx(dev)
ft = th.randn(n, H, D, device=dev)
el = th.randn(n, H, device=dev)
er = th.randn(n, H, device=dev)
out = th.empty(n, H, D, device=dev)
mx = th.empty(n, H, device=dev)
sm = th.empty(n, H, device=dev)
go = th.randn(n, H, D, device=dev)
gft, gel, ger = th.empty_like(ft), th.empty_like(el), th.empty_like(er)
res = {}
# round 3: chunk size only (U = 8 is fixed in the kernels), with the automatic
# column blocks (8 on C3: each launch walks ~14 M edges, ~7000 waves at K = 512)
ks = sys.argv[1].split(",") if len(sys.argv) > 1 else ["128", "256", "512", "1024"]
for rnd in range(2):
    for k in ks:
        os.environ["DGLMI_CHUNK_EDGES"] = k
        f = ev_time(lambda: K.fused_gat_forward(gidx, ft, el, er, 0.2, out, mx, sm))
        b = ev_time(lambda: K.fused_gat_backward(gidx, ft, el, er, 0.2, out, mx, sm, go, gft, gel, ger))
        res.setdefault("K%s" % k, []).append((f, b))
summary = {key: {"fwd_ms": min(x[0] for x in v), "bwd_ms": min(x[1] for x in v)} for key, v in res.items()}
print(json.dumps(summary, indent=1))
