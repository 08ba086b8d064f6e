"""Builtin message functions (``python/dgl/function/message.py``).

Same names, fields and ``name`` strings as the reference: ``copy_u`` /
``copy_src``, ``copy_e`` / ``copy_edge``, ``src_mul_edge`` and the generated
``{u,v,e}_{add,sub,mul,div,dot}_{u,v,e}`` family (``message.py:101-302``).
``_invoke`` goes straight to the backend operator (``F.binary_reduce`` /
``F.copy_reduce``) instead of emitting the reference's mini-IR
(``message.py:47-94``, ``runtime/ir/executor.py:1000-1247``): with both
functions builtin, the reference's scheduler lowers exactly to one such call.
"""
from __future__ import annotations

import sys
from itertools import product

from .base import BuiltinFunction, TargetCode
from .. import backend as B

__all__ = ["src_mul_edge", "copy_src", "copy_edge", "copy_u", "copy_e"]


class MessageFunction(BuiltinFunction):
    """Base builtin message function class."""

    def _invoke(self, gidx, src_frame, dst_frame, edge_frame, out_size, src_map=None,
                dst_map=None, edge_map=None, out_map=None, reducer="none"):
        raise NotImplementedError


def _pair(m):
    return (None, None) if m is None else m


class BinaryMessageFunction(MessageFunction):
    """``lhs_op_rhs`` message (``message.py:30-68``)."""

    def __init__(self, binary_op, lhs, rhs, lhs_field, rhs_field, out_field):
        self.binary_op = binary_op
        self.lhs = lhs
        self.rhs = rhs
        self.lhs_field = lhs_field
        self.rhs_field = rhs_field
        self.out_field = out_field

    def _invoke(self, gidx, src_frame, dst_frame, edge_frame, out_size, src_map=None,
                dst_map=None, edge_map=None, out_map=None, reducer="none"):
        in_frames = (src_frame, dst_frame, edge_frame)
        in_maps = (src_map, dst_map, edge_map)
        lhs_data = in_frames[self.lhs][self.lhs_field]
        rhs_data = in_frames[self.rhs][self.rhs_field]
        return B.binary_reduce(reducer, self.binary_op, gidx, self.lhs, self.rhs, lhs_data,
                               rhs_data, out_size, _pair(in_maps[self.lhs]),
                               _pair(in_maps[self.rhs]), _pair(out_map))

    @property
    def name(self):
        lhs = TargetCode.CODE2STR[self.lhs]
        rhs = TargetCode.CODE2STR[self.rhs]
        return "{}_{}_{}".format(lhs, self.binary_op, rhs)


class CopyMessageFunction(MessageFunction):
    """``copy_*`` message (``message.py:71-98``)."""

    def __init__(self, target, in_field, out_field):
        self.target = target
        self.in_field = in_field
        self.out_field = out_field

    def _invoke(self, gidx, src_frame, dst_frame, edge_frame, out_size, src_map=None,
                dst_map=None, edge_map=None, out_map=None, reducer="none"):
        in_frames = (src_frame, dst_frame, edge_frame)
        in_maps = (src_map, dst_map, edge_map)
        in_data = in_frames[self.target][self.in_field]
        return B.copy_reduce(reducer, gidx, self.target, in_data, out_size,
                             _pair(in_maps[self.target]), _pair(out_map))

    @property
    def name(self):
        return "copy_{}".format(TargetCode.CODE2STR[self.target])


def copy_u(u, out):
    """Message = source node feature ``u`` (``edges.src[u]``)."""
    return CopyMessageFunction(TargetCode.SRC, u, out)


def copy_e(e, out):
    """Message = edge feature ``e`` (``edges.data[e]``)."""
    return CopyMessageFunction(TargetCode.EDGE, e, out)


_TARGET_MAP = {"u": TargetCode.SRC, "v": TargetCode.DST, "e": TargetCode.EDGE}


def _gen_message_builtin(lhs, rhs, binary_op):
    name = "{}_{}_{}".format(lhs, binary_op, rhs)
    docstring = ("Builtin message function that computes a message by performing binary "
                 "operation {} between the {} feature and the {} feature.".format(
                     binary_op, lhs, rhs))

    def func(lhs_field, rhs_field, out):
        return BinaryMessageFunction(binary_op, _TARGET_MAP[lhs], _TARGET_MAP[rhs], lhs_field,
                                     rhs_field, out)

    func.__name__ = name
    func.__doc__ = docstring
    return func


def _register_builtin_message_func():
    target = ["u", "v", "e"]
    for lhs, rhs in product(target, target):
        if lhs != rhs:
            for binary_op in ["add", "sub", "mul", "div", "dot"]:
                func = _gen_message_builtin(lhs, rhs, binary_op)
                setattr(sys.modules[__name__], func.__name__, func)
                __all__.append(func.__name__)


_register_builtin_message_func()


def src_mul_edge(src, edge, out):
    """Deprecated alias of ``u_mul_e``."""
    return getattr(sys.modules[__name__], "u_mul_e")(src, edge, out)


def copy_src(src, out):
    """Deprecated alias of ``copy_u``."""
    return copy_u(src, out)


def copy_edge(edge, out):
    """Deprecated alias of ``copy_e``."""
    return copy_e(edge, out)
