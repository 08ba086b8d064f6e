"""Feature initializers (``python/dgl/init.py``): called as
``initializer(shape, dtype, ctx, id_range)`` for rows a frame must fill itself --
rows of new nodes / edges, rows of a new column outside the written ones, and the
reduce output of zero-in-degree nodes under a reduce UDF
(``runtime/degree_bucketing.py:73-79``)."""
import torch as th

__all__ = ["base_initializer", "zero_initializer"]


def base_initializer(shape, dtype, ctx, id_range):
    raise NotImplementedError


def zero_initializer(shape, dtype, ctx, id_range):
    return th.zeros(shape, dtype=dtype, device=ctx)
