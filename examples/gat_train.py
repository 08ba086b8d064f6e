#!/usr/bin/env python3
"""GAT node classification (the reference's examples/pytorch/gat/gat.py +
train.py: 8 heads x 8 hidden, 1 output head) on the synthetic Cora stand-in.

  python examples/gat_train.py [--epochs 200] [--unfused]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dgl-hack_amd"), os.path.join(ROOT, "examples")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch as th  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dgl  # noqa: E402
from dgl.nn.pytorch import GATConv  # noqa: E402
from _synthetic import planted_cora  # noqa: E402


class GAT(nn.Module):
    """examples/pytorch/gat/gat.py: hidden layers concatenate heads, the output
    layer averages them."""

    def __init__(self, g, in_dim, num_hidden, num_classes, heads, feat_drop, attn_drop,
                 negative_slope, fused):
        super(GAT, self).__init__()
        self.g = g
        self.layers = nn.ModuleList([
            GATConv(in_dim, num_hidden, heads[0], feat_drop, attn_drop, negative_slope,
                    False, F.elu),
            GATConv(num_hidden * heads[0], num_classes, heads[-1], feat_drop, attn_drop,
                    negative_slope, False, None)])
        for layer in self.layers:
            layer.use_fused = fused

    def forward(self, x):
        h = self.layers[0](self.g, x).flatten(1)
        return self.layers[1](self.g, h).mean(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--unfused", action="store_true")
    args = ap.parse_args()
    dev = "cuda:0"
    th.manual_seed(0)
    src, dst, n, x, y, (tr, va, te) = planted_cora(seed=1)
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    g.add_edges(g.nodes(), g.nodes())
    x, y, tr, te = x.to(dev), y.to(dev), tr.to(dev), te.to(dev)
    # attention dropout 0 so the fused kernel serves training too
    model = GAT(g, x.shape[1], 8, int(y.max()) + 1, [8, 1], 0.6, 0.0, 0.2,
                not args.unfused).to(dev)
    opt = th.optim.Adam(model.parameters(), lr=5e-3, weight_decay=5e-4)
    times = []
    for epoch in range(args.epochs):
        model.train()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        loss = F.cross_entropy(model(x)[tr], y[tr])
        opt.zero_grad()
        loss.backward()
        opt.step()
        th.cuda.synchronize()
        if epoch >= 3:
            times.append(time.perf_counter() - t0)
    model.eval()
    with th.no_grad():
        acc = (model(x)[te].argmax(1) == y[te]).float().mean().item()
    print(json.dumps({"example": "gat", "fused": not args.unfused, "epochs": args.epochs,
                      "final_loss": float(loss), "test_acc": acc,
                      "ms_per_epoch": 1e3 * float(np.mean(times)) if times else None}))


if __name__ == "__main__":
    main()
