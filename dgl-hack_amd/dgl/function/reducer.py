"""Builtin reduce functions (``python/dgl/function/reducer.py:28-96``)."""
from __future__ import annotations

import sys

from .base import BuiltinFunction

__all__ = []


class ReduceFunction(BuiltinFunction):
    """Base builtin reduce function class."""


class SimpleReduceFunction(ReduceFunction):
    """Builtin reduce function (``reducer.py:28-49``)."""

    def __init__(self, name, msg_field, out_field):
        self._name = name
        self.msg_field = msg_field
        self.out_field = out_field

    @property
    def name(self):
        return self._name


def _gen_reduce_builtin(reducer):
    def func(msg, out):
        return SimpleReduceFunction(reducer, msg, out)
    func.__name__ = reducer
    func.__doc__ = "Builtin reduce function that aggregates messages by {}.".format(reducer)
    return func


def _register_builtin_reduce_func():
    for reduce_op in ["max", "min", "sum", "prod", "mean"]:
        builtin = _gen_reduce_builtin(reduce_op)
        setattr(sys.modules[__name__], reduce_op, builtin)
        __all__.append(reduce_op)


_register_builtin_reduce_func()
