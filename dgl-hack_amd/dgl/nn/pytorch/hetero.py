"""HeteroGraphConv (``python/dgl/nn/pytorch/hetero.py:18-200``).

Applies one module per relation of a heterograph (each sees the relation as a
bipartite DGLGraph: ``g[stype, etype, dtype]``) and aggregates the results
that land on the same destination type with ``sum`` / ``max`` / ``min`` /
``mean`` / ``stack`` -- same signature and semantics as the reference.
"""
import torch as th
from torch import nn

from ..._ffi import DGLError

__all__ = ["HeteroGraphConv"]


def get_aggregate_fn(agg):
    """hetero.py:172-200: cross-type aggregator over a list of tensors."""
    if agg == "stack":
        return lambda alist, dsttype: th.stack(alist, dim=1)
    ops = {"sum": lambda t: th.sum(t, dim=0), "mean": lambda t: th.mean(t, dim=0),
           "max": lambda t: th.max(t, dim=0)[0], "min": lambda t: th.min(t, dim=0)[0]}
    if agg not in ops:
        raise DGLError("Invalid cross type aggregator. Must be one of sum, max, min, mean or "
                       "stack. But got \"%s\"" % agg)
    op = ops[agg]

    def fn(alist, dsttype):
        if len(alist) == 0:
            return None
        if len(alist) == 1:
            return alist[0]
        return op(th.stack(alist, dim=0))
    return fn


class HeteroGraphConv(nn.Module):
    def __init__(self, mods, aggregate="sum"):
        super(HeteroGraphConv, self).__init__()
        self.mods = nn.ModuleDict(mods)
        self.agg_fn = get_aggregate_fn(aggregate) if isinstance(aggregate, str) else aggregate

    def forward(self, g, inputs, mod_args=None, mod_kwargs=None):
        mod_args = mod_args or {}
        mod_kwargs = mod_kwargs or {}
        outputs = {nty: [] for nty in g.dsttypes}
        pair = isinstance(inputs, tuple)
        src_inputs, dst_inputs = inputs if pair else (inputs, inputs)
        for stype, etype, dtype in g.canonical_etypes:
            rel = g[stype, etype, dtype]
            if rel.number_of_edges() == 0 or stype not in src_inputs:
                continue
            if pair and dtype not in dst_inputs:
                continue
            x = (src_inputs[stype], dst_inputs[dtype]) if pair else src_inputs[stype]
            outputs[dtype].append(self.mods[etype](rel, x, *mod_args.get(etype, ()),
                                                   **mod_kwargs.get(etype, {})))
        return {nty: self.agg_fn(alist, nty) for nty, alist in outputs.items() if alist}
