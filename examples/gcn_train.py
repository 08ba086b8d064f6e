#!/usr/bin/env python3
"""2-layer GCN node classification (the reference's examples/pytorch/gcn/gcn.py +
train.py) on the synthetic Cora stand-in, on one MI355X.

  python examples/gcn_train.py [--epochs 200] [--hidden 16]
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
from dgl.nn.pytorch import GraphConv  # noqa: E402
from _synthetic import planted_cora  # noqa: E402


class GCN(nn.Module):
    """examples/pytorch/gcn/gcn.py:12-40."""

    def __init__(self, g, in_feats, n_hidden, n_classes, n_layers, activation, dropout):
        super(GCN, self).__init__()
        self.g = g
        self.layers = nn.ModuleList([GraphConv(in_feats, n_hidden, activation=activation)])
        for _ in range(n_layers - 1):
            self.layers.append(GraphConv(n_hidden, n_hidden, activation=activation))
        self.layers.append(GraphConv(n_hidden, n_classes))
        self.dropout = nn.Dropout(p=dropout)

    def forward(self, features):
        h = features
        for i, layer in enumerate(self.layers):
            if i != 0:
                h = self.dropout(h)
            h = layer(self.g, h)
        return h


def evaluate(model, features, labels, mask):
    model.eval()
    with th.no_grad():
        logits = model(features)[mask]
        return (logits.argmax(1) == labels[mask]).float().mean().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--hidden", type=int, default=16)
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--weight-decay", type=float, default=5e-4)
    ap.add_argument("--dropout", type=float, default=0.5)
    args = ap.parse_args()
    dev = "cuda:0"
    th.manual_seed(0)
    src, dst, n, x, y, (tr, va, te) = planted_cora()
    g = dgl.DGLGraph()
    g.add_nodes(n)
    g.add_edges(src, dst)
    g.add_edges(g.nodes(), g.nodes())  # self-loops, as train.py does
    x, y, tr, va, te = x.to(dev), y.to(dev), tr.to(dev), va.to(dev), te.to(dev)
    model = GCN(g, x.shape[1], args.hidden, int(y.max()) + 1, args.layers, F.relu,
                args.dropout).to(dev)
    opt = th.optim.Adam(model.parameters(), lr=args.lr, weight_decay=args.weight_decay)
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
    res = {"example": "gcn", "epochs": args.epochs, "final_loss": float(loss),
           "val_acc": evaluate(model, x, y, va), "test_acc": evaluate(model, x, y, te),
           "ms_per_epoch": 1e3 * float(np.mean(times)) if times else None,
           "edges": g.number_of_edges()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
