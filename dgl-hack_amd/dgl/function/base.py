"""Builtin function base classes (``python/dgl/function/base.py:7-40``)."""
from __future__ import annotations


class BuiltinFunction(object):
    """Base builtin function class."""

    @property
    def name(self):
        """Return the name of this builtin function."""
        raise NotImplementedError


class TargetCode(object):
    """Code for target (``function/base.py:7-21``)."""
    SRC = 0
    DST = 1
    EDGE = 2

    CODE2STR = {
        0: "u",
        1: "v",
        2: "e",
    }
