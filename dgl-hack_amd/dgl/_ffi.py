"""ctypes binding of libdglmi.so (the C ABI in include/dglmi.h).

Mirrors the reference's FFI conventions (``python/dgl/_ffi/base.py``):
the library is loaded once with ``RTLD_GLOBAL`` (:31-43, search path
``DGL_LIBRARY_PATH`` like ``_ffi/libinfo.py:32-33``), and every call goes
through :func:`check_call`, which raises :class:`DGLError` with the
library's thread-local last error when a function returns non-zero
(:50-62).  There is no fallback: if the HIP library is missing, importing
the kernel layer fails loudly.
"""
from __future__ import annotations

import ctypes
import os

MAX_NDIM = 8


class DGLError(Exception):
    """Error raised by the engine (python/dgl/_ffi/base.py:24)."""


class CSR(ctypes.Structure):
    _fields_ = [
        ("num_rows", ctypes.c_int64),
        ("num_cols", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("indptr", ctypes.c_void_p),
        ("indices", ctypes.c_void_p),
        ("data", ctypes.c_void_p),
        ("rows", ctypes.c_void_p),
    ]


class Graph(ctypes.Structure):
    _fields_ = [
        ("in_csr", CSR),
        ("out_csr", CSR),
        ("num_bits", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("workspace", ctypes.c_void_p),
        ("workspace_bytes", ctypes.c_int64),
        ("coo_src", ctypes.c_void_p),
        ("coo_dst", ctypes.c_void_p),
        ("in_gather_cols", ctypes.c_void_p),
        ("out_gather_cols", ctypes.c_void_p),
        ("num_col_blocks", ctypes.c_int32),
        ("in_col_blocks", ctypes.c_void_p),
        ("out_col_blocks", ctypes.c_void_p),
        ("rgcn", ctypes.c_void_p),
        ("gat_edge_pos", ctypes.c_void_p),
        ("etypes", ctypes.c_void_p),
        ("eid_identity", ctypes.c_int32),
    ]


class RgcnState(ctypes.Structure):
    """DGLMIRgcnState (include/dglmi.h): per-graph R-GCN state, library-owned."""
    _fields_ = [
        ("etypes", ctypes.c_void_p),
        ("norm", ctypes.c_void_p),
        ("num_rels", ctypes.c_int32),
        ("layers", ctypes.c_int32),
        ("num_src", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("positions", ctypes.c_void_p),
        ("in_cols", ctypes.c_void_p * 2),
        ("in_norm", ctypes.c_void_p),
        ("out_typed", CSR * 2),
        ("out_norm", ctypes.c_void_p * 2),
        ("in_rel", CSR),
        ("in_rel_norm", ctypes.c_void_p),
        ("owner", ctypes.c_void_p),
    ]


class Epilogue(ctypes.Structure):
    _fields_ = [
        ("row_mul", ctypes.c_void_p),
        ("row_div", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("addend", ctypes.c_void_p),
    ]


class DropoutDraw(ctypes.Structure):
    """DGLMIDropoutDraw (include/dglmi.h): torch's fused dropout draw, as launched."""
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("offset", ctypes.c_uint64),
        ("threads", ctypes.c_int64),
        ("vec", ctypes.c_int32),
        ("keep", ctypes.c_float),
        ("scale", ctypes.c_float),
    ]


class Array(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("ndim", ctypes.c_int32),
        ("shape", ctypes.c_int64 * (MAX_NDIM + 1)),
    ]


def _lib_name():
    """libdglmi.so, or with DGLMI_PROBES=1 the probe build libdglmi_probes.so
    (`make -C dgl-hack_amd PROBES=1`: the headline kernel's cache-policy and
    tuning variants, selected by scripts/policy_probe.py / tune_spmm.py through
    the environment; the shipped library has none of them)."""
    return "libdglmi_probes.so" if os.environ.get("DGLMI_PROBES") == "1" else "libdglmi.so"


def _lib_path():
    env = os.environ.get("DGL_LIBRARY_PATH")
    name = _lib_name()
    cands = []
    if env:
        cands.append(os.path.join(env, name))
    cands.append(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", name))
    for c in cands:
        if os.path.exists(c):
            return c
    raise DGLError(
        "%s not found (looked in %s). Build it with `make -C dgl-hack_amd` or "
        "__graft_entry__.build(); the engine has no CPU fallback." % (name, ", ".join(cands)))


_LIB = None

_SIGS = {
    "DGLMIGetLastError": (ctypes.c_char_p, []),
    "DGLMIVersion": (ctypes.c_char_p, []),
    "DGLMISetSddmmOrder": (ctypes.c_int, [ctypes.c_int32]),
    "DGLMIKernelInferBinaryFeatureShape": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]),
    "DGLMIKernelBinaryOpReduce": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIKernelBinaryOpReduceEx": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Epilogue),
        ctypes.c_void_p]),
    "DGLMIKernelCopyReduceEx": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Epilogue),
        ctypes.c_void_p]),
    "DGLMIKernelBackwardLhsBinaryOpReduce": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIKernelBackwardRhsBinaryOpReduce": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIKernelCopyReduce": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIKernelBackwardCopyReduce": (ctypes.c_int, [
        ctypes.c_char_p, ctypes.POINTER(Graph), ctypes.c_int32, ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIKernelWorkspaceBytes": (ctypes.c_int64, [ctypes.POINTER(CSR), ctypes.c_int64]),
    "DGLMIKernelMarkColdColumns": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMICOOToCSR": (ctypes.c_int, [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMICSRTranspose": (ctypes.c_int, [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMICOOToCSRDeviceWorkspaceBytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
    "DGLMICOOToCSRDevice": (ctypes.c_int, [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
        ctypes.c_void_p]),
    "DGLMIFusedGatSupported": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64]),
    "DGLMIFusedGatForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIFusedGatBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIFusedGatForwardEx": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIFusedGatBackwardEx": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIFusedGatDropoutForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.c_float, ctypes.c_uint64, ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIFusedGatDropoutBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.c_float, ctypes.c_uint64, ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIFusedGatKeepForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIFusedGatKeepBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIFusedGatDrawForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(DropoutDraw),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIFusedGatDrawBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(DropoutDraw),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIDropoutDrawMask": (ctypes.c_int, [
        ctypes.POINTER(DropoutDraw), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIDropoutDrawScale": (ctypes.c_int, [
        ctypes.POINTER(DropoutDraw), ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
        ctypes.c_void_p]),
    "DGLMIDropoutDrawApply": (ctypes.c_int, [
        ctypes.POINTER(DropoutDraw), ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
        ctypes.c_void_p]),
    "DGLMIGatKeepGather": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
        ctypes.c_void_p]),
    "DGLMIGatKeepBits": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
        ctypes.c_void_p]),
    "DGLMIGatKeepBitsMask": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
        ctypes.c_void_p]),
    "DGLMIFusedGatKernel": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_float,
        ctypes.c_void_p]),
    "DGLMIKernelBackwardFusedGat": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_float,
        ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxSupported": (ctypes.c_int, [ctypes.c_int64]),
    "DGLMIEdgeSoftmaxWorkspaceBytes": (ctypes.c_int64, [ctypes.POINTER(CSR), ctypes.c_int64]),
    "DGLMIEdgeSoftmaxForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxNodeLogitsForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_float,
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxNodeLogitsForwardEx": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_float,
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxNodeLogitsBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_float, ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIProjectSupported": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64]),
    "DGLMIProject": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_int, ctypes.c_void_p]),
    "DGLMIGatAttnLogitsSupported": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64]),
    "DGLMIGatAttnLogitsPartials": (ctypes.c_int64, [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]),
    "DGLMIGatAttnLogits": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
        ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_int, ctypes.c_void_p]),
    "DGLMIGatAttnLogitsBackward": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
        ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "DGLMIGatherRows": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
        ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxLeakyForward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.c_float, ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIEdgeSoftmaxLeakyBackward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_float, ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIPartitionLDG": (ctypes.c_int, [
        ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_double,
        ctypes.c_void_p]),
    "DGLMICSRExpandRows": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMICSRExpandRows64": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMICOOToCSRDevice64WorkspaceBytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
    "DGLMICOOToCSRDevice64": (ctypes.c_int, [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
        ctypes.c_void_p]),
    "DGLMIPartitionLabelProp": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_void_p,
        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "DGLMIRgcnLayer0": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIRgcnLayer0Backward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIRgcnLayer1": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIRgcnLayer1Ex": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Epilogue),
        ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIRgcnLayer1BackwardEx": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.c_void_p]),
    "DGLMIRgcnLayer1Backward": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array), ctypes.POINTER(Array),
        ctypes.c_void_p]),
    "DGLMIRgcnPrepare": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.c_int32,
        ctypes.c_int32, ctypes.POINTER(RgcnState), ctypes.c_void_p]),
    "DGLMIRgcnRefreshNorm": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.POINTER(RgcnState), ctypes.c_void_p]),
    "DGLMIRgcnRelease": (ctypes.c_int, [ctypes.POINTER(RgcnState)]),
    "DGLMINbAccess": (ctypes.c_int, [
        ctypes.POINTER(Graph), ctypes.POINTER(Array), ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p]),
    "DGLMIStreamCopy": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
}

EXPORTED = tuple(_SIGS)


def lib():
    """The loaded library (loaded on first use)."""
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(_lib_path(), mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def last_error():
    return lib().DGLMIGetLastError().decode()


def check_call(ret):
    """Raise DGLError if a C ABI call failed (python/dgl/_ffi/base.py:50-62)."""
    if ret != 0:
        raise DGLError(last_error())
