"""UDF / degree-bucketing restatement -- TEST INFRASTRUCTURE ONLY.

The reference's kernel tests never compare builtins against stored numbers;
they compare them against the same computation expressed as user-defined
message/reduce functions, which DGL executes by materialising every message
and reducing per destination node in degree buckets
(``python/dgl/runtime/degree_bucketing.py:12-…``,
``tests/compute/test_kernel.py:225-290``).  This module restates that path
with plain torch CPU ops in float64 (autograd gives the gradients), so the C
oracle and the HIP kernels are both checked against an independent
formulation.

Zero-in-degree nodes are reported as NaN here: the UDF path never writes
them, while the builtin path writes the reducer identity
(``binary_reduce_impl.h:62``); tests compare those rows separately.
"""
from __future__ import annotations

import numpy as np
import torch as th

SRC, DST, EDGE = "u", "v", "e"


def _align(a, b):
    # tests/compute/test_kernel.py:254-259 -- batched broadcast by unsqueezing dim 1
    while a.dim() < b.dim():
        a = a.unsqueeze(1)
    while b.dim() < a.dim():
        b = b.unsqueeze(1)
    return a, b


def message(op, lhs_e, rhs_e):
    if rhs_e is None:
        return lhs_e
    a, b = _align(lhs_e, rhs_e)
    if op == "add":
        return a + b
    if op == "sub":
        return a - b
    if op == "mul":
        return a * b
    if op == "div":
        return a / b
    if op == "dot":
        return (a * b).sum(-1)
    raise ValueError(op)


def _gather(t, target, src, dst):
    if target == SRC:
        return t[src]
    if target == DST:
        return t[dst]
    return t  # edge data is already per edge (eid order)


def degree_bucket_reduce(msg, dst, num_nodes, reducer):
    """Reduce per-edge messages (eid order) into destination nodes by degree bucket."""
    dst_np = dst.numpy()
    order = np.argsort(dst_np, kind="stable")
    deg = np.bincount(dst_np, minlength=num_nodes)
    starts = np.concatenate([[0], np.cumsum(deg)])
    out = th.full((num_nodes,) + tuple(msg.shape[1:]), float("nan"), dtype=msg.dtype)
    rows = []
    vals = []
    for d in np.unique(deg):
        if d == 0:
            continue
        nodes = np.nonzero(deg == d)[0]
        idx = np.stack([order[starts[v]:starts[v] + d] for v in nodes])  # (nb, d)
        mailbox = msg[th.from_numpy(idx)]  # (nb, d, ...)
        if reducer == "sum":
            r = mailbox.sum(1)
        elif reducer == "max":
            r = mailbox.max(1)[0]
        elif reducer == "min":
            r = mailbox.min(1)[0]
        elif reducer == "prod":
            r = mailbox.prod(1)
        elif reducer == "mean":
            r = mailbox.mean(1)
        else:
            raise ValueError(reducer)
        rows.append(th.from_numpy(nodes))
        vals.append(r)
    if rows:
        out = out.index_put((th.cat(rows),), th.cat(vals))
    return out


def update_all(src, dst, num_nodes, lhs_t, rhs_t, op, reducer, data, grad=True):
    """Builtin-equivalent UDF pipeline.  `data` maps 'u','v','e' -> float64 tensors.

    Returns (result, {target: grad}) with grads of sum(result over non-NaN rows).
    """
    src_t = th.as_tensor(np.asarray(src), dtype=th.long)
    dst_t = th.as_tensor(np.asarray(dst), dtype=th.long)
    leaves = {k: v.detach().clone().double().requires_grad_(grad) for k, v in data.items()}
    lhs_e = _gather(leaves[lhs_t], lhs_t, src_t, dst_t)
    rhs_e = None if rhs_t is None else _gather(leaves[rhs_t], rhs_t, src_t, dst_t)
    msg = message(op, lhs_e, rhs_e)
    if reducer == "none":
        res = msg
    else:
        res = degree_bucket_reduce(msg, dst_t, num_nodes, reducer)
    grads = {}
    if grad:
        mask = ~th.isnan(res)
        th.where(mask, res, th.zeros_like(res)).sum().backward()
        grads = {k: (v.grad if v.grad is not None else th.zeros_like(v)) for k, v in leaves.items()}
    return res.detach(), grads
