#!/usr/bin/env python3
"""Which summation order torch's (x * a).sum(-1) uses on this device for an innermost
dimension of D = 4 .. 64 (GATConv's el / er): bit-match fraction of candidate orders,
each evaluated with explicit fp32 additions of the rounded products."""
import json

import torch as th

DEV = "cuda:0"
g = th.Generator(device=DEV).manual_seed(0)


def seq(p):
    s = p[..., 0]
    for i in range(1, p.shape[-1]):
        s = s + p[..., i]
    return s


def tree(p):
    while p.shape[-1] > 1:
        p = p[..., 0::2] + p[..., 1::2]
    return p[..., 0]


def acc_w(p, w, comb):
    # w accumulators, element i into accumulator i % w, then combined by `comb`
    a = p[..., 0:w].clone()
    for j in range(w, p.shape[-1], w):
        a = a + p[..., j:j + w]
    return comb(a)


def halves(p):
    # butterfly over lanes holding consecutive quads: quad sums sequential, then a tree
    q = seq(p.view(*p.shape[:-1], -1, 4).transpose(-1, -2).transpose(-1, -2)) if False else None
    s = [seq(p[..., i:i + 4]) for i in range(0, p.shape[-1], 4)]
    t = th.stack(s, -1)
    return tree(t)


for D in (4, 8, 16, 32, 64):
    x = th.randn(200000, 8, D, device=DEV, generator=g)
    a = th.randn(1, 8, D, device=DEV, generator=g)
    ref = (x * a).sum(-1)
    p = x * a
    cands = {"seq": seq(p), "tree": tree(p), "quads_then_tree(kernel)": halves(p)}
    for w in (2, 4, 8):
        if w < D:
            cands["acc%d_seq" % w] = acc_w(p, w, seq)
            cands["acc%d_tree" % w] = acc_w(p, w, tree)
    out = {"D": D}
    for k, v in cands.items():
        out[k] = float((v == ref).float().mean())
    print(json.dumps(out), flush=True)
