#!/usr/bin/env python3
"""GATConv's fused route with the device el / er (gatconv.FUSED_ATTN_LOGITS) against
torch's multiply + sum: per-tensor max differences of the output and every gradient for
a few (H, D) shapes, with and without attention dropout (debug / A-B probe)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch as th  # noqa: E402

import dgl  # noqa: E402
from dgl.nn.pytorch import GATConv  # noqa: E402
from dgl.nn.pytorch.conv import gatconv  # noqa: E402
from graphs import powerlaw  # noqa: E402

DEV = "cuda:0"
src, dst, n = powerlaw(20000, 300000, seed=22)
g = dgl.DGLGraph()
g.add_nodes(n)
g.add_edges(src, dst)
for H, D, p in ((32, 4, 0.0), (32, 4, 0.6), (8, 8, 0.6), (16, 4, 0.0), (4, 8, 0.0)):
    conv = GATConv(24, D, H, attn_drop=p).to(DEV).train()
    x0 = th.randn(n, 24, device=DEV, generator=th.Generator(device=DEV).manual_seed(2))
    go = th.randn(n, H, D, device=DEV, generator=th.Generator(device=DEV).manual_seed(3))
    res = []
    for flag in (True, False):
        gatconv.FUSED_ATTN_LOGITS = flag
        conv.zero_grad()
        x = x0.clone().requires_grad_()
        th.manual_seed(11)
        y = conv(g, x)
        y.backward(go)
        res.append((y.detach(), x.grad, conv.fc.weight.grad.clone(), conv.attn_l.grad.clone(),
                    conv.attn_r.grad.clone()))
    out = {"H": H, "D": D, "p": p}
    for a, b, name in zip(res[0], res[1], ("y", "x", "fc", "attn_l", "attn_r")):
        out[name] = [float((a - b).abs().max()), float(b.abs().max())]
    print(json.dumps(out), flush=True)
