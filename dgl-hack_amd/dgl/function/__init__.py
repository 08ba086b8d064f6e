"""Builtin message and reduce functions (``dgl.function``)."""
from .base import BuiltinFunction, TargetCode
from .message import *  # noqa: F401,F403
from .reducer import *  # noqa: F401,F403
