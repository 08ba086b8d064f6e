"""Kernel wrappers over the C ABI (mirrors ``python/dgl/kernel.py``).

Every function takes the per-device graph index (``ImmutableGraphIndex``),
torch tensors on that device and optional int32 mapping tensors, and runs on
torch's current HIP stream.  The output / gradient buffers are caller-owned
and overwritten completely, exactly like the reference's
``K.binary_op_reduce`` family (``kernel.py:29-436``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch as th

from . import _ffi
from ._ffi import DGLError, check_call

_TARGET = {"src": 0, "dst": 1, "edge": 2, "none": 3}


def _arr(t, name):
    if t is None:
        return None
    if not isinstance(t, th.Tensor):
        raise DGLError("%s must be a torch tensor" % name)
    if t.device.type != "cuda":
        raise DGLError("%s is on %s: the MI355X engine runs on ROCm devices only" % (name, t.device))
    if t.dtype != th.float32:
        raise DGLError("Unsupported dtype: %s for %s (float32 only, kernel/common.h:49-55)" % (t.dtype, name))
    if not t.is_contiguous():
        raise DGLError("%s must be contiguous" % name)
    if t.dim() > _ffi.MAX_NDIM + 1:
        raise DGLError("%s has too many dimensions" % name)
    a = _ffi.Array()
    a.data = t.data_ptr() if t.numel() else None
    a.ndim = t.dim() if t.dim() > 0 else 1
    shape = list(t.shape) if t.dim() > 0 else [1]
    for i, s in enumerate(shape):
        a.shape[i] = s
    a._keep = t
    return ctypes.byref(a)


_KEEP_BITS = {th.uint8: 8, th.int16: 16, th.int32: 32}


def _keep_words(t, name, num_edges):
    """(pointer, bits) of a keep-word tensor: contiguous 1-D uint8 / int16 / int32 on the
    device, one word per edge."""
    if not isinstance(t, th.Tensor) or t.device.type != "cuda" or t.dtype not in _KEEP_BITS \
            or not t.is_contiguous() or t.dim() != 1 or t.shape[0] != num_edges:
        raise DGLError("%s must be a contiguous (E,) uint8 / int16 / int32 ROCm tensor" % name)
    return ctypes.c_void_p(t.data_ptr() if t.numel() else None), _KEEP_BITS[t.dtype]


def _map(m, name):
    if m is None:
        return None
    if not isinstance(m, th.Tensor) or m.dtype != th.int32 or m.device.type != "cuda":
        raise DGLError("Expected 32 integer array on the graph device for %s" % name)
    return ctypes.c_void_p(m.contiguous().data_ptr())


def _stream(t):
    return ctypes.c_void_p(th.cuda.current_stream(t.device).cuda_stream)


def _check_ctx(graph, tensors):
    for name, t in tensors:
        if t is not None and t.device != graph.device:
            raise DGLError("Expected device context %s. But got %s for %s." % (graph.device, t.device, name))


def _workspace(graph, feat_len, device):
    nbytes = graph.workspace_bytes(feat_len)
    if nbytes <= 0:
        return None
    return th.empty(int(nbytes), dtype=th.uint8, device=device)


def spmm_col_blocks(graph, feat_len):
    """Column blocks for the load-balanced sums (DGLMIGraph.num_col_blocks): when
    the gathered node table fits the Infinity Cache but not L2 (32-256 MiB) and
    rows are long (average in-degree >= 64, so chaining per-block partial sums is
    cheap), one pass per block of ~8 MiB of table (a power of two <= 32).
    Reddit-size graph (114.6 M edges; scripts/spmm_block_probe.py,
    profiles/r01_spmm_blocks.json), chained passes included: copy_u_sum F = 64
    3.88 -> 2.96 ms (8 blocks), F = 128 7.99 -> 4.70 ms (16 blocks).  The library
    applies them to copy_u sums only.  DGLMI_SPMM_BLOCKS overrides (1 = off)."""
    env = os.environ.get("DGLMI_SPMM_BLOCKS")
    if env is not None:
        return max(1, int(env))
    ic = graph.in_csr
    table = ic.num_cols * feat_len * 4
    if not ((32 << 20) <= table < (256 << 20)) or ic.nnz < (1 << 22) or ic.nnz < 64 * max(1, ic.num_rows):
        return 1
    nb = 1
    while nb < 32 and table / nb > (8 << 20):
        nb *= 2
    return nb


def _cgraph(graph, ws, per_edge, feat_len=0):
    """Graph struct for a call; per-edge outputs also get the edge-id ordered COO;
    reductions over a large-degree graph get its column blocks."""
    nb = spmm_col_blocks(graph, feat_len) if feat_len and not per_edge else 1
    return graph.cstruct(ws, coo=per_edge, col_blocks=nb)


def _feat_len(t):
    n = 1
    for s in t.shape[1:]:
        n *= s
    return n


def infer_binary_feature_shape(op, lhs, rhs):
    """kernel.py:8-26 / binary_reduce.cc:281-293 (host-only shape logic)."""
    def mk(t):
        a = _ffi.Array()
        a.data = None
        shape = list(t.shape)
        a.ndim = len(shape)
        for i, s in enumerate(shape):
            a.shape[i] = s
        return a
    la, ra = mk(lhs), mk(rhs)
    out = (ctypes.c_int64 * (_ffi.MAX_NDIM + 1))()
    nd = ctypes.c_int32(0)
    check_call(_ffi.lib().DGLMIKernelInferBinaryFeatureShape(
        op.encode(), ctypes.byref(la), ctypes.byref(ra), out, ctypes.byref(nd)))
    return tuple(out[i] for i in range(nd.value))


def _epilogue(epilogue, out_data):
    """(row_mul, row_div, bias[, addend]) float32 tensors on out's device (None allowed)."""
    if epilogue is None or all(t is None for t in epilogue):
        return None
    e = _ffi.Epilogue()
    keep = []
    names = ("row_mul", "row_div", "bias", "addend")
    for name in names[len(epilogue):]:
        setattr(e, name, None)
    for name, t in zip(names, epilogue):
        if t is None:
            setattr(e, name, None)
            continue
        t = t.contiguous()
        if t.dtype != th.float32 or t.device != out_data.device:
            raise DGLError("epilogue %s must be float32 on %s" % (name, out_data.device))
        want = {"bias": _feat_len(out_data), "addend": out_data.numel()}.get(name, out_data.shape[0])
        if t.numel() != want:
            raise DGLError("epilogue %s has %d values, expected %d" % (name, t.numel(), want))
        if name == "addend":
            lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * 4
            olo, ohi = out_data.data_ptr(), out_data.data_ptr() + out_data.numel() * 4
            if lo < ohi and olo < hi:
                raise DGLError("epilogue addend must not overlap the output")
        setattr(e, name, t.data_ptr())
        keep.append(t)
    e._keep = keep
    return e


def binary_op_reduce(reducer, op, graph, lhs, rhs, lhs_data, rhs_data, out_data,
                     lhs_map=None, rhs_map=None, out_map=None, epilogue=None):
    """kernel.py:29-148 -> _CAPI_DGLKernelBinaryOpReduce.  ``epilogue`` =
    (row_mul, row_div, bias) fused into a "sum" reduction (DGLMIKernelBinaryOpReduceEx)."""
    _check_ctx(graph, [("lhs_data", lhs_data), ("rhs_data", rhs_data), ("out_data", out_data)])
    ws = _workspace(graph, _feat_len(out_data), out_data.device)
    g = _cgraph(graph, ws, reducer == "none", _feat_len(out_data))
    epi = _epilogue(epilogue, out_data)
    args = (reducer.encode(), op.encode(), ctypes.byref(g), _TARGET_CODE(lhs), _TARGET_CODE(rhs),
            _arr(lhs_data, "lhs_data"), _arr(rhs_data, "rhs_data"), _arr(out_data, "out_data"),
            _map(lhs_map, "lhs_mapping"), _map(rhs_map, "rhs_mapping"),
            _map(out_map, "out_mapping"))
    if epi is None:
        check_call(_ffi.lib().DGLMIKernelBinaryOpReduce(*args, _stream(out_data)))
    else:
        check_call(_ffi.lib().DGLMIKernelBinaryOpReduceEx(*args, ctypes.byref(epi),
                                                          _stream(out_data)))
    return out_data


def backward_lhs_binary_op_reduce(reducer, op, graph, lhs, rhs, lhs_data, rhs_data, out_data,
                                  grad_out_data, grad_lhs_data, lhs_map=None, rhs_map=None,
                                  out_map=None):
    """kernel.py:151-229 -> _CAPI_DGLKernelBackwardLhsBinaryOpReduce."""
    _check_ctx(graph, [("lhs_data", lhs_data), ("rhs_data", rhs_data), ("out_data", out_data),
                       ("grad_out_data", grad_out_data), ("grad_lhs_data", grad_lhs_data)])
    ws = _workspace(graph, _feat_len(grad_lhs_data), grad_lhs_data.device)
    g = _cgraph(graph, ws, _TARGET_CODE(lhs) == 2, _feat_len(grad_lhs_data))
    check_call(_ffi.lib().DGLMIKernelBackwardLhsBinaryOpReduce(
        reducer.encode(), op.encode(), ctypes.byref(g), _TARGET_CODE(lhs), _TARGET_CODE(rhs),
        _map(lhs_map, "lhs_mapping"), _map(rhs_map, "rhs_mapping"), _map(out_map, "out_mapping"),
        _arr(lhs_data, "lhs_data"), _arr(rhs_data, "rhs_data"), _arr(out_data, "out_data"),
        _arr(grad_out_data, "grad_out_data"), _arr(grad_lhs_data, "grad_lhs_data"),
        _stream(grad_lhs_data)))
    return grad_lhs_data


def backward_rhs_binary_op_reduce(reducer, op, graph, lhs, rhs, lhs_data, rhs_data, out_data,
                                  grad_out_data, grad_rhs_data, lhs_map=None, rhs_map=None,
                                  out_map=None):
    """kernel.py:232-299 -> _CAPI_DGLKernelBackwardRhsBinaryOpReduce."""
    _check_ctx(graph, [("lhs_data", lhs_data), ("rhs_data", rhs_data), ("out_data", out_data),
                       ("grad_out_data", grad_out_data), ("grad_rhs_data", grad_rhs_data)])
    ws = _workspace(graph, _feat_len(grad_rhs_data), grad_rhs_data.device)
    g = _cgraph(graph, ws, _TARGET_CODE(rhs) == 2, _feat_len(grad_rhs_data))
    check_call(_ffi.lib().DGLMIKernelBackwardRhsBinaryOpReduce(
        reducer.encode(), op.encode(), ctypes.byref(g), _TARGET_CODE(lhs), _TARGET_CODE(rhs),
        _map(lhs_map, "lhs_mapping"), _map(rhs_map, "rhs_mapping"), _map(out_map, "out_mapping"),
        _arr(lhs_data, "lhs_data"), _arr(rhs_data, "rhs_data"), _arr(out_data, "out_data"),
        _arr(grad_out_data, "grad_out_data"), _arr(grad_rhs_data, "grad_rhs_data"),
        _stream(grad_rhs_data)))
    return grad_rhs_data


def copy_reduce(reducer, graph, target, in_data, out_data, in_map=None, out_map=None,
                epilogue=None):
    """kernel.py:302-393 -> _CAPI_DGLKernelCopyReduce (``epilogue``: see binary_op_reduce)."""
    _check_ctx(graph, [("in_data", in_data), ("out_data", out_data)])
    ws = _workspace(graph, _feat_len(out_data), out_data.device)
    g = _cgraph(graph, ws, reducer == "none", _feat_len(out_data))
    epi = _epilogue(epilogue, out_data)
    args = (reducer.encode(), ctypes.byref(g), _TARGET_CODE(target), _arr(in_data, "in_data"),
            _arr(out_data, "out_data"), _map(in_map, "in_mapping"), _map(out_map, "out_mapping"))
    if epi is None:
        check_call(_ffi.lib().DGLMIKernelCopyReduce(*args, _stream(out_data)))
    else:
        check_call(_ffi.lib().DGLMIKernelCopyReduceEx(*args, ctypes.byref(epi), _stream(out_data)))
    return out_data


def backward_copy_reduce(reducer, graph, target, in_data, out_data, grad_out_data, grad_in_data,
                         in_map=None, out_map=None):
    """kernel.py:396-436 -> _CAPI_DGLKernelBackwardCopyReduce."""
    _check_ctx(graph, [("in_data", in_data), ("out_data", out_data),
                       ("grad_out_data", grad_out_data), ("grad_in_data", grad_in_data)])
    ws = _workspace(graph, _feat_len(grad_in_data), grad_in_data.device)
    g = _cgraph(graph, ws, _TARGET_CODE(target) == 2, _feat_len(grad_in_data))
    check_call(_ffi.lib().DGLMIKernelBackwardCopyReduce(
        reducer.encode(), ctypes.byref(g), _TARGET_CODE(target), _arr(in_data, "in_data"),
        _arr(out_data, "out_data"), _arr(grad_out_data, "grad_out_data"),
        _arr(grad_in_data, "grad_in_data"), _map(in_map, "in_mapping"),
        _map(out_map, "out_mapping"), _stream(grad_in_data)))
    return grad_in_data


_SDDMM_ORDERS = {"auto": 0, "coo": 1, "csr": 2}


def set_sddmm_order(order):
    """Item order of the per-edge (g-SDDMM) kernels, process-wide: "auto" (the
    library picks per call), "coo" (edge-id order) or "csr"
    (in-CSR order) -- DGLMISetSddmmOrder; tests and probes cover both walks."""
    check_call(_ffi.lib().DGLMISetSddmmOrder(_SDDMM_ORDERS[order]))


def _TARGET_CODE(t):
    if isinstance(t, str):
        return _TARGET[t]
    return int(t)


def fused_gat_supported(heads, head_dim):
    return bool(_ffi.lib().DGLMIFusedGatSupported(int(heads), int(head_dim)))


def fused_gat_head_dim(heads, head_dim):
    """Head width the fused GAT kernel runs at: ``head_dim`` itself, or the
    smallest supported width above it (zero-padded columns aggregate to zero and
    are sliced off -- e.g. a 41-class output layer runs at 64 instead of falling
    back to the generic kernels); None if no width up to 1024 / heads works."""
    d = int(head_dim)
    if fused_gat_supported(heads, d):
        return d
    c = 4
    while heads * c <= 1024:
        if c >= d and fused_gat_supported(heads, c):
            return c
        c += 4
    return None


def gat_col_blocks(graph, feat_src, backward=False):
    """Column blocks for the fused GAT kernels (DGLMIGraph.num_col_blocks): when the
    gathered ft + el table fits the Infinity Cache but not L2 (>= 32 MiB) and rows
    are long (average in-degree >= 64, so merging per-block row partials is cheap),
    cut the sources into blocks of 6-12 MiB of table each (a power of two <= 16),
    the same count for the forward and both backward walks (one set of block CSRs).
    C3 (67 MB table; scripts/gat_ab.py + scripts/gpu_gat_prof.sh,
    profiles/r02_gat_blocks.json): forward 5.8 ms whole / 4.38 (4 blocks) / 3.43 (8)
    / 3.66 (16); backward 12.0 / 9.86 (4) / 9.00 (8) / 9.59 (16).
    DGLMI_GAT_BLOCKS overrides (1 = off).  `backward` is kept for callers."""
    env = os.environ.get("DGLMI_GAT_BLOCKS")
    if env is not None:
        return max(1, int(env))
    n_src = feat_src.shape[0]
    h = feat_src.shape[1] if feat_src.dim() == 3 else 1
    table = n_src * (_feat_len(feat_src) + h) * 4
    nnz, rows = graph.in_csr.nnz, max(1, graph.in_csr.num_rows)
    if table < (32 << 20) or nnz < (1 << 22) or nnz < 64 * rows:
        return 1
    target = 6 << 20
    nb = 1
    while nb < 16 and table / (nb * 2) >= target:
        nb *= 2
    return nb


def gat_edge_pos(graph, col_blocks):
    """Whether the fused GAT backward takes the edge-position path (DGLMIGraph
    .gat_edge_pos: no destination-side walk; grad_er from the source-side walk's
    per-edge terms): unblocked whole graphs (edge ids a permutation).  C3 unblocked
    11.98 -> 9.57 ms, M1-size RMAT 11.48 -> 10.89 ms; with column blocks the
    destination walk stays faster (8.52 vs 9.15 ms; profiles/r03_gat_edge_pos.json).
    DGLMI_GAT_EDGE_POS=0 keeps the destination-side walk."""
    return (os.environ.get("DGLMI_GAT_EDGE_POS", "1") != "0" and graph.eid_perm
            and col_blocks <= 1)


def _gat_bwd_cgraph(graph, feat_src):
    nb = gat_col_blocks(graph, feat_src, backward=True)
    return graph.cstruct(None, col_blocks=nb, edge_pos=gat_edge_pos(graph, nb))


def gat_dropout_keep(seed, eids, num_heads, p):
    """The fused GAT's attention-dropout mask (DGLMIFusedGatDropout*; internal.h
    gat_edge_key / gat_pair_bits / gat_head_keep) on the host, for tests: a
    (len(eids), num_heads) bool array, True where edge eids[i], head h keeps its weight.
    One key per edge (a mix of the edge id and the seed), one multiply-xorshift per pair
    of heads whose low / high 16 bits decide the two heads against round(p 2^16).  numpy uint32 arithmetic wraps like the kernel's."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)

    def mix(x):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846CA68B)
        return x ^ (x >> np.uint32(16))
    def finish(x):  # gat_pair_bits: one multiply
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        return x ^ (x >> np.uint32(15))
    e = np.asarray(eids, dtype=np.int64).astype(np.uint32)
    pairs = (num_heads + 1) // 2
    with np.errstate(over="ignore"):
        key = mix(e ^ lo) ^ hi
        off = (np.arange(pairs, dtype=np.uint32) + np.uint32(1)) * np.uint32(0x9E3779B9)
        r = finish(key[:, None] + off[None, :])                   # (E, pairs)
    u16 = np.stack([r & np.uint32(0xFFFF), r >> np.uint32(16)], 2).reshape(len(e), 2 * pairs)
    return u16[:, :num_heads].astype(np.int64) >= _gat_drop_thresh(p)


def _gat_drop_thresh(p):
    """The C entry's 16-bit threshold round(p 2^16), capped at 2^16 (keeps nothing)."""
    return min(65536, int(np.floor(float(np.float32(p)) * 65536.0 + 0.5)))


def gat_dropout_scale(p):
    """The hashed mask's scale for kept weights (capi.cpp gat_set_dropout): the inverse of
    the quantised keep probability (2^16 - t) / 2^16, so E[dropout(a)] = a exactly; 0
    when nothing is kept."""
    t = _gat_drop_thresh(p)
    return float(np.float32(65536.0 / (65536.0 - t))) if t < 65536 else 0.0


def gat_keep_bits(table):
    """One keep word per edge from a dropout output ``table`` (E, H[, 1]) float32 or the
    dropout's boolean mask (torch.native_dropout's second output) in edge-id order: bit h
    set where head h was kept (non-zero / True), in the narrowest word that holds H (uint8
    for H <= 8, int16 for H <= 16, int32 for H <= 32) -> DGLMIGatKeepBits[Mask]."""
    h = 1
    for d in table.shape[1:]:
        h *= int(d)
    t = table.reshape(table.shape[0], h)
    is_mask = t.dtype == th.bool
    if not (is_mask or t.dtype == th.float32) or not t.is_cuda:
        raise DGLError("gat_keep_bits: a float32 table or a bool mask on the ROCm device")
    t = t.contiguous()
    h = int(t.shape[1])
    if not 1 <= h <= 32:
        raise DGLError("gat_keep_bits: 1 <= heads <= 32")
    dt, width = (th.uint8, 8) if h <= 8 else (th.int16, 16) if h <= 16 else (th.int32, 32)
    bits = th.empty(t.shape[0], dtype=dt, device=t.device)
    if is_mask and h == 8 and t.data_ptr() % 8:
        t = t.clone()  # the 8-head path reads a row as one 8-byte word
    entry = _ffi.lib().DGLMIGatKeepBitsMask if is_mask else _ffi.lib().DGLMIGatKeepBits
    check_call(entry(ctypes.c_void_p(t.data_ptr() if t.numel() else None), ctypes.c_int64(t.shape[0]), h,
                     ctypes.c_void_p(bits.data_ptr() if bits.numel() else None), width, _stream(bits)))
    return bits


def gat_keep_walk_order(graph, keep, feat_src, direction):
    """The keep words (edge-id order) in the position order of the fused GAT's walks over
    ``graph`` for ``feat_src``: "in" the forward's (the in-CSR, or its column blocks in
    block order), "out" the backward's (the out-CSR or its blocks) -> DGLMIGatKeepGather
    per block.  With these the kernels read one coalesced word per position instead of a
    random one per edge (DGLMIFusedGatKeep*, keep_by_position)."""
    nb = gat_col_blocks(graph, feat_src)
    if nb > 1:
        ib, ob = graph.col_blocks(nb)
        csrs = ib if direction == "in" else ob
    else:
        csrs = [graph.in_csr if direction == "in" else graph.out_csr]
    out = th.empty_like(keep)
    kp, kb = _keep_words(keep, "keep", graph.in_csr.nnz)
    off = 0
    for c in csrs:
        n = int(c.nnz)
        if n:
            idx = c.data
            if idx.dtype != th.int32 or not idx.is_contiguous():
                raise DGLError("gat_keep_walk_order: int32 edge ids expected")
            check_call(_ffi.lib().DGLMIGatKeepGather(
                kp, kb, ctypes.c_void_p(idx.data_ptr()), ctypes.c_int64(n),
                ctypes.c_void_p(out.data_ptr() + off * out.element_size()), _stream(out)))
        off += n
    if off != keep.shape[0]:
        raise DGLError("gat_keep_walk_order: the walk covers %d of %d edges" % (off, keep.shape[0]))
    return out


def dropout_draw(device, numel, p):
    """Take torch's fused dropout draw for a contiguous float32 tensor of ``numel``
    elements on ``device`` with drop probability 0 < ``p`` < 1, as nn.Dropout(p) would:
    the generator's Philox offset advances by the draws per thread (the kernel's 256-thread
    blocks, grid capped at CUs x maxThreadsPerCU / 256, four uniforms a draw), and the
    returned DGLMIDropoutDraw lets the fused GAT kernels recompute every element's keep
    decision (DGLMIFusedGatDraw*).  Not under stream capture (the generator's captured
    offsets are device-side); callers check :func:`dropout_draw_ok` first."""
    dev = th.device(device)
    props = th.cuda.get_device_properties(dev)
    blocks = props.multi_processor_count * (props.max_threads_per_multi_processor // 256)
    grid = min(blocks, (numel + 255) // 256)
    inc = ((numel - 1) // (256 * grid * 4) + 1) * 4
    gen = th.cuda.default_generators[dev.index if dev.index is not None else th.cuda.current_device()]
    seed, off = gen.initial_seed(), gen.get_offset()
    gen.set_offset(off + inc)
    vec = 4 if numel % 4 == 0 else 2 if numel % 2 == 0 else 1
    keep = np.float32(1.0 - float(p))
    return _ffi.DropoutDraw(seed & 0xFFFFFFFFFFFFFFFF, off, grid * 256, vec, float(keep),
                            float(np.float32(1.0 / float(keep))))


def dropout_draw_mask(draw, numel, device):
    """The draw's whole keep mask (bool, ``numel``) -> DGLMIDropoutDrawMask."""
    out = th.empty(numel, dtype=th.uint8, device=device)
    check_call(_ffi.lib().DGLMIDropoutDrawMask(
        ctypes.byref(draw), ctypes.c_int64(numel), ctypes.c_void_p(out.data_ptr() if numel else None),
        _stream(out)))
    return out.bool()


def dropout_draw_scale(draw, heads, eids, num_edges, device):
    """(E, heads, 1) float32: the draw's output on ones -- draw.scale where kept, else 0 --
    at position p for edge ``eids[p]`` (int32 ROCm tensor; None = identity) ->
    DGLMIDropoutDrawScale.  The same values as ``nn.Dropout(p)(ones)[eids]`` from the
    generator state the draw was taken at."""
    out = th.empty((num_edges, heads, 1), dtype=th.float32, device=device)
    if eids is not None and (eids.dtype != th.int32 or not eids.is_contiguous() or eids.numel() != num_edges):
        raise DGLError("dropout_draw_scale: eids must be a contiguous int32 tensor of E ids")
    check_call(_ffi.lib().DGLMIDropoutDrawScale(
        ctypes.byref(draw), int(heads), ctypes.c_void_p(eids.data_ptr() if eids is not None and num_edges else None),
        ctypes.c_int64(num_edges), ctypes.c_void_p(out.data_ptr() if num_edges else None), _stream(out)))
    return out


def dropout_draw_apply(draw, heads, eids, x):
    """x (E, heads[, 1]) float32 contiguous, in place: x *= draw.scale where kept, else 0,
    at position p for edge ``eids[p]`` -> DGLMIDropoutDrawApply.  Returns x."""
    n = x.shape[0]
    if not (x.is_cuda and x.dtype == th.float32 and x.is_contiguous() and x.numel() == n * heads):
        raise DGLError("dropout_draw_apply: a contiguous float32 (E, heads) ROCm tensor")
    if eids is not None and (eids.dtype != th.int32 or not eids.is_contiguous() or eids.numel() != n):
        raise DGLError("dropout_draw_apply: eids must be a contiguous int32 tensor of E ids")
    check_call(_ffi.lib().DGLMIDropoutDrawApply(
        ctypes.byref(draw), int(heads), ctypes.c_void_p(eids.data_ptr() if eids is not None and n else None),
        ctypes.c_int64(n), ctypes.c_void_p(x.data_ptr() if n else None), _stream(x)))
    return x


_DRAW_OK = {}


def dropout_draw_ok(device):
    """Whether :func:`dropout_draw` reproduces torch.native_dropout on this device and
    build: checked once per device against torch itself -- the masks of a vec-4 draw with
    the grid capped, vec-2 and vec-1 draws, and the generator offset each leaves -- with
    the generator state restored afterwards.  False under stream capture."""
    dev = th.device(device)
    if dev.type != "cuda" or th.cuda.is_current_stream_capturing():
        return False
    idx = dev.index if dev.index is not None else th.cuda.current_device()
    if idx not in _DRAW_OK:
        gen = th.cuda.default_generators[idx]
        state = gen.get_state()
        ok = True
        try:
            for n in ((1 << 23) + 8, 2002, 3003, 2 * ((1 << 21) + 1)):
                gen.manual_seed(1234 + n)
                d = dropout_draw(dev, n, 0.6)
                after = gen.get_offset()
                gen.manual_seed(1234 + n)
                _, m = th.native_dropout(th.empty(n, device=dev), 0.6, True)
                ok = ok and gen.get_offset() == after and bool(th.equal(dropout_draw_mask(d, n, dev), m))
        finally:
            gen.set_state(state)
        _DRAW_OK[idx] = ok
    return _DRAW_OK[idx]


def fused_gat_forward(graph, feat_src, el, er, slope, out, max_out, sum_out, slope_feat=None,
                      slope_sum=None, attn_drop=0.0, seed=0, keep=None, keep_scale=None,
                      keep_pos=False, draw=None):
    """_CAPI_DGLFusedGatKernel (binary_reduce.cc:380-396) -> DGLMIFusedGatForward, or
    with ``slope_feat`` (N, H, D) / ``slope_sum`` (N, H) DGLMIFusedGatForwardEx: the
    forward also keeps the attention's slope aggregates, so the backward needs no
    destination-side walk.  ``attn_drop`` > 0: DGLMIFusedGatDropoutForward (GATConv's
    attention dropout in the same pass, the mask a hash of ``seed`` and the edge id).
    ``keep`` (E,) keep words (:func:`gat_keep_bits`) with ``keep_scale``:
    DGLMIFusedGatKeepForward, the caller's mask -- by edge id, or with ``keep_pos`` in the
    forward walk's position order (:func:`gat_keep_walk_order` "in").  ``draw``
    (:func:`dropout_draw`): DGLMIFusedGatDrawForward, torch's own draws recomputed."""
    _check_ctx(graph, [("feat_src", feat_src), ("el", el), ("er", er), ("out", out)])
    g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src))
    if draw is not None:
        check_call(_ffi.lib().DGLMIFusedGatDrawForward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), ctypes.byref(draw), _arr(out, "out"), _arr(max_out, "max_out"),
            _arr(sum_out, "sum_out"), _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"),
            _stream(out)))
        return out
    if keep is not None:
        kp, kb = _keep_words(keep, "keep", graph.in_csr.nnz)
        check_call(_ffi.lib().DGLMIFusedGatKeepForward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), kp, kb, int(bool(keep_pos)), float(keep_scale), _arr(out, "out"),
            _arr(max_out, "max_out"), _arr(sum_out, "sum_out"), _arr(slope_feat, "slope_feat"),
            _arr(slope_sum, "slope_sum"), _stream(out)))
        return out
    if attn_drop > 0.0:
        check_call(_ffi.lib().DGLMIFusedGatDropoutForward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), float(attn_drop), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF),
            _arr(out, "out"), _arr(max_out, "max_out"), _arr(sum_out, "sum_out"),
            _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"), _stream(out)))
        return out
    args = [ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), _arr(out, "out"), _arr(max_out, "max_out"), _arr(sum_out, "sum_out")]
    if slope_feat is None:
        check_call(_ffi.lib().DGLMIFusedGatForward(*args, _stream(out)))
    else:
        check_call(_ffi.lib().DGLMIFusedGatForwardEx(
            *args, _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"), _stream(out)))
    return out


def fused_gat_backward(graph, feat_src, el, er, slope, out, max_in, sum_in, grad_out,
                       grad_feat_src, grad_el, grad_er, slope_feat=None, slope_sum=None,
                       attn_drop=0.0, seed=0, keep=None, keep_scale=None, keep_pos=False,
                       draw=None):
    """_CAPI_DGLKernelBackwardFusedGat (binary_reduce.cc:529-549) -> DGLMIFusedGatBackward
    (or DGLMIFusedGatBackwardEx with the forward's slope aggregates; with ``attn_drop`` > 0
    DGLMIFusedGatDropoutBackward, the forward's seed; with ``keep``
    DGLMIFusedGatKeepBackward, the forward's mask -- by edge id, or with ``keep_pos`` in the
    backward walk's position order, :func:`gat_keep_walk_order` "out"; with ``draw``
    DGLMIFusedGatDrawBackward, the forward's draw)."""
    _check_ctx(graph, [("feat_src", feat_src), ("grad_out", grad_out)])
    if draw is not None:  # without slope aggregates: the destination-side walks recompute too
        g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src, backward=True))
        check_call(_ffi.lib().DGLMIFusedGatDrawBackward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), ctypes.byref(draw), _arr(out, "out"), _arr(max_in, "max_in"),
            _arr(sum_in, "sum_in"), _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"),
            _arr(grad_out, "grad_out"), _arr(grad_feat_src, "grad_feat_src"), _arr(grad_el, "grad_el"),
            _arr(grad_er, "grad_er"), _stream(grad_out)))
        return
    if keep is not None:
        if slope_feat is None:
            raise DGLError("fused GAT dropout backward needs the forward's slope aggregates")
        g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src, backward=True))
        kp, kb = _keep_words(keep, "keep", graph.in_csr.nnz)
        check_call(_ffi.lib().DGLMIFusedGatKeepBackward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), kp, kb, int(bool(keep_pos)), float(keep_scale), _arr(out, "out"),
            _arr(max_in, "max_in"), _arr(sum_in, "sum_in"), _arr(slope_feat, "slope_feat"),
            _arr(slope_sum, "slope_sum"), _arr(grad_out, "grad_out"),
            _arr(grad_feat_src, "grad_feat_src"), _arr(grad_el, "grad_el"),
            _arr(grad_er, "grad_er"), _stream(grad_out)))
        return
    if attn_drop > 0.0:
        if slope_feat is None:
            raise DGLError("fused GAT dropout backward needs the forward's slope aggregates")
        g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src, backward=True))
        check_call(_ffi.lib().DGLMIFusedGatDropoutBackward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), float(attn_drop), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF),
            _arr(out, "out"), _arr(max_in, "max_in"), _arr(sum_in, "sum_in"),
            _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"),
            _arr(grad_out, "grad_out"), _arr(grad_feat_src, "grad_feat_src"),
            _arr(grad_el, "grad_el"), _arr(grad_er, "grad_er"), _stream(grad_out)))
        return
    if slope_feat is None:
        g = _gat_bwd_cgraph(graph, feat_src)
        check_call(_ffi.lib().DGLMIFusedGatBackward(
            ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"),
            float(slope), _arr(out, "out"), _arr(max_in, "max_in"), _arr(sum_in, "sum_in"),
            _arr(grad_out, "grad_out"), _arr(grad_feat_src, "grad_feat_src"),
            _arr(grad_el, "grad_el"), _arr(grad_er, "grad_er"), _stream(grad_out)))
        return
    g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src, backward=True))
    check_call(_ffi.lib().DGLMIFusedGatBackwardEx(
        ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"), float(slope),
        _arr(out, "out"), _arr(max_in, "max_in"), _arr(sum_in, "sum_in"),
        _arr(slope_feat, "slope_feat"), _arr(slope_sum, "slope_sum"),
        _arr(grad_out, "grad_out"), _arr(grad_feat_src, "grad_feat_src"), _arr(grad_el, "grad_el"),
        _arr(grad_er, "grad_er"), _stream(grad_out)))


def fused_gat_kernel(graph, feat_src, el, er, s, exp, ret, slope):
    """The reference's ``kernel.fused_gat_kernel`` (kernel.py:150-151) in its own
    argument order: _CAPI_DGLFusedGatKernel (binary_reduce.cc:380-396) ->
    DGLMIFusedGatKernel.  ``s`` (N, H[, 1]) and ``exp`` (E, H[, 1]) are the
    caller's buffers carrying the softmax state to :func:`backward_fused_gat`."""
    _check_ctx(graph, [("feat_src", feat_src), ("el", el), ("er", er), ("s", s), ("exp", exp),
                       ("ret", ret)])
    g = graph.cstruct(None, col_blocks=gat_col_blocks(graph, feat_src))
    check_call(_ffi.lib().DGLMIFusedGatKernel(
        ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"), _arr(s, "s"),
        _arr(exp, "exp"), _arr(ret, "ret"), float(slope), _stream(ret)))
    return ret


def backward_fused_gat(graph, feat_src, el, er, s, exp, ret, grad_out, grad_feat_src, grad_el,
                       grad_er, slope):
    """The reference's ``kernel.backward_fused_gat`` (kernel.py:153-154):
    _CAPI_DGLKernelBackwardFusedGat (binary_reduce.cc:529-549) ->
    DGLMIKernelBackwardFusedGat.  Overwrites the three gradients."""
    _check_ctx(graph, [("feat_src", feat_src), ("grad_out", grad_out)])
    g = _gat_bwd_cgraph(graph, feat_src)
    check_call(_ffi.lib().DGLMIKernelBackwardFusedGat(
        ctypes.byref(g), _arr(feat_src, "feat_src"), _arr(el, "el"), _arr(er, "er"), _arr(s, "s"),
        _arr(exp, "exp"), _arr(ret, "ret"), _arr(grad_out, "grad_out"),
        _arr(grad_feat_src, "grad_feat_src"), _arr(grad_el, "grad_el"), _arr(grad_er, "grad_er"),
        float(slope), _stream(grad_out)))


def edge_softmax_supported(values_per_edge):
    return bool(_ffi.lib().DGLMIEdgeSoftmaxSupported(int(values_per_edge)))


def _softmax_ws(graph, h, device):
    nbytes = _ffi.lib().DGLMIEdgeSoftmaxWorkspaceBytes(ctypes.byref(graph.in_csr.cstruct()), int(h))
    return th.empty(int(nbytes), dtype=th.uint8, device=device) if nbytes > 0 else None


def edge_softmax_forward(graph, logits, out):
    """Fused edge softmax (extension of softmax.py:15-84) -> DGLMIEdgeSoftmaxForward."""
    _check_ctx(graph, [("logits", logits), ("out", out)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(logits), logits.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxForward(ctypes.byref(g), _arr(logits, "logits"),
                                                  _arr(out, "out"), _stream(out)))
    return out


def edge_softmax_backward(graph, out, grad_out, grad_logits):
    """softmax.py:86-114 fused -> DGLMIEdgeSoftmaxBackward."""
    _check_ctx(graph, [("out", out), ("grad_out", grad_out), ("grad_logits", grad_logits)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(out), out.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxBackward(ctypes.byref(g), _arr(out, "out"),
                                                   _arr(grad_out, "grad_out"),
                                                   _arr(grad_logits, "grad_logits"), _stream(out)))
    return grad_logits


# projections on the MFMA kernel from this many rows (fewer: torch.matmul, launch-bound)
PROJECT_MIN_ROWS = 1 << 14


def project_mfma_ok(x2, w):
    """Whether Y = x2 @ w runs on DGLMIProject: fp32 ROCm tensors on one device, x2 a
    contiguous (M, K) matrix with M >= PROJECT_MIN_ROWS whose K equals w's row count
    (a mismatch stays on torch.matmul, which raises), (K, N) supported."""
    return (x2.is_cuda and x2.dtype == th.float32 and w.dtype == th.float32 and w.dim() == 2
            and x2.dim() == 2 and w.device == x2.device and x2.is_contiguous()
            and x2.shape[1] == w.shape[0]
            and x2.shape[0] >= PROJECT_MIN_ROWS and x2.data_ptr() % 16 == 0
            and w.stride(0) >= 1 and w.stride(1) >= 1
            and bool(_ffi.lib().DGLMIProjectSupported(int(w.shape[0]), int(w.shape[1]))))


def project_bias_ok(b, n, device):
    """Whether ``b`` can ride in DGLMIProject's epilogue: an fp32 vector of the output
    width on the device whose contiguous form is 16-byte aligned (a slice of a flat
    parameter buffer may not be; it then takes torch.addmm)."""
    if not (b.dim() == 1 and b.dtype == th.float32 and b.shape[0] == n and b.device == device):
        return False
    return b.contiguous().data_ptr() % 16 == 0


def project_mfma(x2, w, bias=None):
    """x2 @ w (+ bias) on the MFMA projection kernel -> DGLMIProject (w may be a
    transposed view; its strides are passed; its row count is checked against x2's
    columns in C)."""
    m, k = x2.shape
    n = int(w.shape[1])
    y = x2.new_empty((m, n))
    if bias is not None:
        bias = bias.contiguous()
    check_call(_ffi.lib().DGLMIProject(
        ctypes.c_void_p(x2.data_ptr()), ctypes.c_int64(m), ctypes.c_int64(k),
        ctypes.c_void_p(w.data_ptr()), ctypes.c_int64(w.shape[0]), ctypes.c_int64(w.stride(0)),
        ctypes.c_int64(w.stride(1)), ctypes.c_int64(n),
        ctypes.c_void_p(bias.data_ptr() if bias is not None else None),
        ctypes.c_void_p(y.data_ptr()), int(x2.device.index or 0), _stream(y)))
    return y


def attn_logits_ok(feat_src, feat_dst, attn_l, attn_r):
    """Whether GATConv's el / er (gatconv.py:137-138) can take DGLMIGatAttnLogits: fp32
    contiguous (N, H, D) features on one ROCm device (16-B aligned) and (1, H, D) attention
    vectors there, (H, D) a supported shape."""
    if not (feat_src.is_cuda and feat_src.dim() == 3 and feat_src.dtype == th.float32):
        return False
    _, h, d = feat_src.shape
    for t in (feat_src, feat_dst):
        if not (t.dim() == 3 and t.shape[1:] == (h, d) and t.dtype == th.float32
                and t.device == feat_src.device and t.is_contiguous() and t.data_ptr() % 16 == 0):
            return False
    for a in (attn_l, attn_r):
        if not (a.shape == (1, h, d) and a.dtype == th.float32 and a.device == feat_src.device):
            return False
    return bool(_ffi.lib().DGLMIGatAttnLogitsSupported(int(h), int(d)))


def _aligned(t):
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def attn_logits(feat_src, feat_dst, attn_l, attn_r):
    """(el, er) of shape (N, H, 1) -> DGLMIGatAttnLogits; ``feat_dst`` None: one table."""
    ns, h, d = feat_src.shape
    nd = ns if feat_dst is None else feat_dst.shape[0]
    el = feat_src.new_empty((ns, h, 1))
    er = feat_src.new_empty((nd, h, 1))
    al, ar = _aligned(attn_l), _aligned(attn_r)
    check_call(_ffi.lib().DGLMIGatAttnLogits(
        ctypes.c_void_p(feat_src.data_ptr()),
        ctypes.c_void_p(None if feat_dst is None else feat_dst.data_ptr()),
        ctypes.c_int64(ns), ctypes.c_int64(nd), ctypes.c_int64(h), ctypes.c_int64(d),
        ctypes.c_void_p(al.data_ptr()), ctypes.c_void_p(ar.data_ptr()),
        ctypes.c_void_p(el.data_ptr()), ctypes.c_void_p(er.data_ptr()),
        int(feat_src.device.index or 0), _stream(el)))
    return el, er


def attn_logits_backward(feat_src, feat_dst, attn_l, attn_r, grad_el, grad_er):
    """-> (grad_src, grad_dst or None, grad_attn_l, grad_attn_r) through
    DGLMIGatAttnLogitsBackward; the parameter gradients sum the per-thread partials of
    each slot in thread order (a fixed grid per shape: deterministic)."""
    ns, h, d = feat_src.shape
    nd = ns if feat_dst is None else feat_dst.shape[0]
    al, ar = _aligned(attn_l), _aligned(attn_r)
    gel, ger = grad_el.contiguous(), grad_er.contiguous()
    gs = th.empty_like(feat_src)
    gd = None if feat_dst is None else th.empty_like(feat_dst)
    nt = int(_ffi.lib().DGLMIGatAttnLogitsPartials(ns, nd, h, d))
    part = feat_src.new_empty((nt, 8))
    check_call(_ffi.lib().DGLMIGatAttnLogitsBackward(
        ctypes.c_void_p(feat_src.data_ptr()),
        ctypes.c_void_p(None if feat_dst is None else feat_dst.data_ptr()),
        ctypes.c_int64(ns), ctypes.c_int64(nd), ctypes.c_int64(h), ctypes.c_int64(d),
        ctypes.c_void_p(al.data_ptr()), ctypes.c_void_p(ar.data_ptr()),
        ctypes.c_void_p(gel.data_ptr()), ctypes.c_void_p(ger.data_ptr()),
        ctypes.c_void_p(gs.data_ptr()), ctypes.c_void_p(None if gd is None else gd.data_ptr()),
        ctypes.c_void_p(part.data_ptr()), int(feat_src.device.index or 0), _stream(gs)))
    f4 = h * d // 4
    p = part.view(nt // f4, f4, 2, 4).sum(0)  # (slot, {l, r}, 4)
    return gs, gd, p[:, 0, :].reshape(1, h, d), p[:, 1, :].reshape(1, h, d)


def gather_rows(src, index, check=False):
    """src[index] for a contiguous fp32 device tensor and an int32 / int64 index on its
    device -> DGLMIGatherRows (one random row read per output row, rows written in
    order); other dtypes take torch's indexing.  The kernel does NOT bound-check:
    every index must lie in [0, src.shape[0]) -- the internal callers pass a CSR's edge
    ids or positions, in range by construction.  ``check=True`` verifies the range
    first (one device reduction and a host sync) and raises DGLError as torch's
    indexing raises IndexError."""
    if src.dtype != th.float32 or index.dtype not in (th.int32, th.int64):
        return src[index.long()]
    if not src.is_cuda or index.device != src.device:
        raise DGLError("gather_rows: src and index must be on one ROCm device")
    if check and index.numel():
        lo, hi = int(index.min()), int(index.max())
        if lo < 0 or hi >= src.shape[0]:
            raise DGLError("gather_rows: index out of range [%d, %d] for %d rows"
                           % (lo, hi, src.shape[0]))
    src = src.contiguous()
    index = index.contiguous()
    out = src.new_empty((index.shape[0],) + tuple(src.shape[1:]))
    row = 1
    for d in src.shape[1:]:
        row *= d
    check_call(_ffi.lib().DGLMIGatherRows(
        ctypes.c_void_p(src.data_ptr()), ctypes.c_int64(row), ctypes.c_void_p(index.data_ptr()),
        32 if index.dtype == th.int32 else 64, ctypes.c_int64(index.shape[0]),
        ctypes.c_void_p(out.data_ptr()), _stream(out)))
    return out


def edge_softmax_node_logits_forward(graph, el, er, negative_slope, out):
    """edge_softmax(leaky_relu(el[u] + er[v])) without stored logits (GATConv's u_add_v,
    leaky_relu, edge_softmax) -> DGLMIEdgeSoftmaxNodeLogitsForward."""
    _check_ctx(graph, [("el", el), ("er", er), ("out", out)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(out), out.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxNodeLogitsForward(
        ctypes.byref(g), _arr(el, "el"), _arr(er, "er"), ctypes.c_float(negative_slope),
        _arr(out, "out"), _stream(out)))
    return out


def edge_softmax_node_logits_forward_ex(graph, el, er, negative_slope, out, row_max, row_sum):
    """edge_softmax_node_logits_forward, also keeping each destination row's (max, sum of
    exp) -> DGLMIEdgeSoftmaxNodeLogitsForwardEx (the fused GAT backward's softmax state)."""
    _check_ctx(graph, [("el", el), ("er", er), ("out", out), ("row_max", row_max),
                       ("row_sum", row_sum)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(out), out.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxNodeLogitsForwardEx(
        ctypes.byref(g), _arr(el, "el"), _arr(er, "er"), ctypes.c_float(negative_slope),
        _arr(out, "out"), _arr(row_max, "row_max"), _arr(row_sum, "row_sum"), _stream(out)))
    return out


def edge_softmax_node_logits_backward(graph, out, grad_out, el, er, negative_slope, grad_logits):
    """The gradient wrt the logits el[u] + er[v] (before leaky_relu) of
    edge_softmax_node_logits_forward -> DGLMIEdgeSoftmaxNodeLogitsBackward."""
    _check_ctx(graph, [("out", out), ("grad_out", grad_out), ("el", el), ("er", er),
                       ("grad_logits", grad_logits)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(out), out.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxNodeLogitsBackward(
        ctypes.byref(g), _arr(out, "out"), _arr(grad_out, "grad_out"), _arr(el, "el"),
        _arr(er, "er"), ctypes.c_float(negative_slope), _arr(grad_logits, "grad_logits"),
        _stream(out)))
    return grad_logits


def edge_softmax_leaky_forward(graph, logits, negative_slope, out):
    """edge_softmax(leaky_relu(logits)) in the softmax's passes (GATConv's pair,
    gatconv.py:160-161) -> DGLMIEdgeSoftmaxLeakyForward; ``logits`` pre-activation."""
    _check_ctx(graph, [("logits", logits), ("out", out)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(logits), logits.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxLeakyForward(ctypes.byref(g), _arr(logits, "logits"),
                                                       ctypes.c_float(negative_slope),
                                                       _arr(out, "out"), _stream(out)))
    return out


def edge_softmax_leaky_backward(graph, out, grad_out, logits, negative_slope, grad_logits):
    """The gradient wrt the pre-activation logits of edge_softmax_leaky_forward ->
    DGLMIEdgeSoftmaxLeakyBackward."""
    _check_ctx(graph, [("out", out), ("grad_out", grad_out), ("logits", logits),
                       ("grad_logits", grad_logits)])
    g = graph.cstruct(_softmax_ws(graph, _feat_len(out), out.device), coo=True)
    check_call(_ffi.lib().DGLMIEdgeSoftmaxLeakyBackward(
        ctypes.byref(g), _arr(out, "out"), _arr(grad_out, "grad_out"), _arr(logits, "logits"),
        ctypes.c_float(negative_slope), _arr(grad_logits, "grad_logits"), _stream(out)))
    return grad_logits


# --------------------------------------------------------------------------- #
# the hack's extra kernels (kernel.py:156-169 of the reference)
# --------------------------------------------------------------------------- #
def _etypes(graph, etypes=None):
    """The relation ids a call uses: ``etypes`` when given, else the graph's own
    (``graph.etypes``, from ``add_edges_with_type``), like the reference's kernels read
    them from the graph object (``graph.cc:690-746``).  int32 on the graph device, one
    entry per edge id."""
    if etypes is None:
        etypes = getattr(graph, "etypes", None)
        if etypes is None:
            raise DGLError("the graph has no edge types (add_edges_with_type) and no etypes "
                           "were given")
    if not isinstance(etypes, th.Tensor) or etypes.dtype != th.int32 or etypes.device != graph.device:
        raise DGLError("etypes must be an int32 tensor on the graph device (one entry per edge id)")
    if etypes.numel() != graph.in_csr.nnz:
        raise DGLError("etypes needs one entry per edge")
    return etypes if etypes.is_contiguous() else etypes.contiguous()


def nb_access(graph, feat, node_map=None, deg_inc_node_map=None, times=15, warm_up_times=5):
    """_CAPI_DGLNbAccess: time `times` in-neighbour row gathers of ``feat``; returns
    the mean microseconds of the launches after the warm-ups."""
    _check_ctx(graph, [("feat", feat)])
    avg = ctypes.c_double(0.0)
    check_call(_ffi.lib().DGLMINbAccess(
        ctypes.byref(graph.cstruct(_workspace(graph, feat[0].numel(), feat.device))),
        _arr(feat, "feat"), _map(node_map, "node_map"), _map(deg_inc_node_map, "deg_inc_node_map"),
        int(times), int(warm_up_times), ctypes.byref(avg), _stream(feat)))
    return avg.value


class RgcnState:
    """A prepared DGLMIRgcnState (DGLMIRgcnPrepare) of one graph for one set of edge
    types: the relation-expanded in-CSR columns, the out-CSR regrouped by (relation,
    source) and the edge weights in both walks' position orders, built once on the
    device.  It holds the etypes and norm tensors, so their memory cannot be reused by
    another tensor while the state lives.  A different or rewritten norm re-gathers
    the cached copies (DGLMIRgcnRefreshNorm: three E-float gathers, no re-sort).
    Released by ``release()`` or with the object."""

    live = 0  # states holding device memory (tests check a rebuild keeps one)

    def __init__(self, graph, norm, num_rels, layers, etypes=None):
        et = _etypes(graph, etypes)
        if norm is not None:
            _check_ctx(graph, [("norm", norm)])
        self.etypes, self.norm = et, norm
        self.versions = (et._version, None if norm is None else norm._version)
        self.num_rels, self.layers = int(num_rels), int(layers)
        self.c = _ffi.RgcnState()
        g = graph.cstruct()
        g.etypes = et.data_ptr()
        check_call(_ffi.lib().DGLMIRgcnPrepare(
            ctypes.byref(g), None if norm is None else _arr(norm, "norm"), self.num_rels,
            self.layers, ctypes.byref(self.c), _stream(et)))
        self._graph_struct = g  # for DGLMIRgcnRefreshNorm (pointers fixed for the graph's life)
        import weakref
        RgcnState.live += 1
        self._fin = weakref.finalize(self, RgcnState._free, self.c)

    @staticmethod
    def _free(c):
        _ffi.lib().DGLMIRgcnRelease(ctypes.byref(c))
        RgcnState.live -= 1

    def release(self):
        """Free the device memory now (DGLMIRgcnRelease)."""
        self._fin()

    def matches(self, etypes, num_rels, layer):
        """True when a call over these relation ids may use the state (the C entries
        compare pointers; the version counter also catches in-place writes, and views
        of the same storage share it)."""
        if not self._fin.alive or etypes.data_ptr() != self.etypes.data_ptr() \
                or etypes.numel() != self.etypes.numel() or etypes._version != self.versions[0]:
            return False
        usable = (self.layers >> layer) & 1 or (layer == 1 and self.layers & 4)
        return int(num_rels) == self.num_rels and bool(usable)

    def sync_norm(self, norm):
        """Before a call with ``norm``: the C side streams the cached copies whenever the
        pointer equals the cached one, so a rewritten (version changed) or new norm is
        re-gathered first."""
        if self.norm is None or norm is None:
            return
        if norm.data_ptr() == self.norm.data_ptr() and norm._version == self.versions[1]:
            return
        flat = norm.reshape(-1)
        if not flat.is_contiguous() or flat.numel() != self.c.nnz:
            return  # read by edge id (the pointer differs from the cached one)
        g = self._graph_struct
        check_call(_ffi.lib().DGLMIRgcnRefreshNorm(ctypes.byref(g), _arr(norm, "norm"),
                                                   ctypes.byref(self.c), _stream(norm)))
        self.norm = norm
        self.versions = (self.versions[0], norm._version)


def rgcn_prepare(graph, norm, num_rels, layers=7, etypes=None):
    """DGLMIRgcnPrepare: build the R-GCN state of ``graph`` for its edge types (or
    ``etypes``: int32, one per edge id) and ``norm`` (one float per edge id, or None)
    once; later rgcn_layer* calls on this graph over the same relation ids use it
    (layers bit 0: Layer0 and its backward, bit 1: Layer1 and its backward, bit 2: the
    fused Layer1 kernels for 64-wide gathered rows -- equal to the unfused path up to
    fp32 rounding).  The graph's previous state is released first, so a rebuild never
    holds two.  Writing into etypes in place invalidates the state (the next call
    derives everything per call); a new or rewritten norm is re-gathered."""
    old = graph.__dict__.pop("_rgcn_state", None)
    if old is not None:
        old.release()
    st = RgcnState(graph, norm, num_rels, layers, etypes)
    graph.__dict__["_rgcn_state"] = st
    return st


def _rgcn_cgraph(graph, etypes, norm, num_rels, layer):
    """The DGLMIGraph of an R-GCN call: the graph's relation ids in ``etypes`` (the
    reference's graph object carries them) and its prepared state when it applies."""
    et = _etypes(graph, etypes)
    g = graph.cstruct()
    g.etypes = et.data_ptr()
    st = graph.__dict__.get("_rgcn_state")
    if st is not None and st.matches(et, num_rels, layer):
        st.sync_norm(norm)
        g.rgcn = ctypes.addressof(st.c)
    return g, et


def rgcn_layer0(graph, weight, norm, ret, etypes=None):
    """_CAPI_DGLRgcnLayer0(G, weight, norm, ret) (kernel.py:159-160 of the reference):
    ret[v] = sum_e weight[etypes[e], u] * norm[e], the relation ids from the graph."""
    _check_ctx(graph, [("weight", weight), ("norm", norm), ("ret", ret)])
    g, et = _rgcn_cgraph(graph, etypes, norm, weight.shape[0], 0)
    check_call(_ffi.lib().DGLMIRgcnLayer0(
        ctypes.byref(g), _arr(weight, "weight"), _arr(norm, "norm"), _arr(ret, "ret"),
        _stream(ret)))


def rgcn_layer0_backward(graph, grad_out, norm, grad_weight, etypes=None):
    """_CAPI_DGLRgcnLayer0Backward(G, grad_out, norm, grad_weight) (exact sums over
    repeated (source, relation) pairs)."""
    _check_ctx(graph, [("grad_out", grad_out), ("norm", norm), ("grad_weight", grad_weight)])
    g, et = _rgcn_cgraph(graph, etypes, norm, grad_weight.shape[0], 0)
    check_call(_ffi.lib().DGLMIRgcnLayer0Backward(
        ctypes.byref(g), _arr(grad_out, "grad_out"), _arr(norm, "norm"),
        _arr(grad_weight, "grad_weight"), _stream(grad_out)))


def rgcn_layer1(graph, x, weight, norm, ret, etypes=None):
    """_CAPI_DGLRgcnLayer1(G, hidden, weight, norm, ret):
    ret[v] = sum_e norm[e] * x[u] . weight[etypes[e]]."""
    _check_ctx(graph, [("hidden", x), ("weight", weight), ("norm", norm), ("ret", ret)])
    g, et = _rgcn_cgraph(graph, etypes, norm, weight.shape[0], 1)
    check_call(_ffi.lib().DGLMIRgcnLayer1(
        ctypes.byref(g), _arr(x, "hidden"), _arr(weight, "weight"), _arr(norm, "norm"),
        _arr(ret, "ret"), _stream(ret)))


def rgcn_layer1_ex(graph, hidden, weight, norm, ret, loop_weight=None, bias=None,
                   addend=None, etypes=None):
    """DGLMIRgcnLayer1Ex: rgcn_layer1 + hidden . loop_weight + bias (+ addend), RelGraphConv's
    self-loop and bias in the same pass (relgraphconv.py:186-190 order)."""
    _check_ctx(graph, [("hidden", hidden), ("weight", weight), ("norm", norm), ("ret", ret),
                       ("loop_weight", loop_weight)])
    epi = _epilogue((None, None, bias, addend), ret)
    if epi is not None and epi.addend and epi.addend % 16:
        raise DGLError("epilogue addend must be 16-byte aligned")
    g, et = _rgcn_cgraph(graph, etypes, norm, weight.shape[0], 1)
    check_call(_ffi.lib().DGLMIRgcnLayer1Ex(
        ctypes.byref(g), _arr(hidden, "hidden"), _arr(weight, "weight"), _arr(norm, "norm"),
        _arr(loop_weight, "loop_weight"), None if epi is None else ctypes.byref(epi),
        _arr(ret, "ret"), _stream(ret)))


def rgcn_layer1_backward_ex(graph, hidden, weight, norm, loop_weight, grad_out,
                            grad_hidden, grad_weight, grad_loop_weight=None, etypes=None):
    """DGLMIRgcnLayer1BackwardEx: rgcn_layer1_backward with the self-loop term in
    grad_hidden, and hidden^T . grad_out into grad_loop_weight (if given)."""
    _check_ctx(graph, [("hidden", hidden), ("weight", weight), ("norm", norm),
                       ("loop_weight", loop_weight), ("grad_out", grad_out),
                       ("grad_hidden", grad_hidden), ("grad_weight", grad_weight),
                       ("grad_loop_weight", grad_loop_weight)])
    g, et = _rgcn_cgraph(graph, etypes, norm, weight.shape[0], 1)
    check_call(_ffi.lib().DGLMIRgcnLayer1BackwardEx(
        ctypes.byref(g), _arr(hidden, "hidden"), _arr(weight, "weight"), _arr(norm, "norm"),
        _arr(loop_weight, "loop_weight"), _arr(grad_out, "grad_out"),
        _arr(grad_hidden, "grad_hidden"), _arr(grad_weight, "grad_weight"),
        _arr(grad_loop_weight, "grad_loop_weight"), _stream(grad_out)))


def rgcn_fused_ok(gathered_w, out_w, num_rels):
    """The shapes the fused layer-1 kernels take (hack_kernels.hip rgcn_fused_ok):
    64-float gathered rows, 1..128 outputs, all weight matrices (``num_rels`` counts the
    self-loop one too) in 80 KB of LDS."""
    if gathered_w != 64 or not 1 <= out_w <= 128 or num_rels < 1:
        return False
    nb = 1 if out_w <= 32 else (2 if out_w <= 64 else 4)
    return num_rels * 64 * nb * 32 <= 20480


def rgcn_layer1_backward(graph, hidden, weight, norm, grad_out, grad_hidden, grad_weight,
                         etypes=None):
    """_CAPI_DGLRgcnLayer1Backward(G, hidden, weight, norm, grad_out, grad_hidden,
    grad_weight): both gradients (the hack's wrapper drops the weight gradient,
    tensor.py:493; it is returned here)."""
    _check_ctx(graph, [("hidden", hidden), ("weight", weight), ("norm", norm),
                       ("grad_out", grad_out), ("grad_hidden", grad_hidden),
                       ("grad_weight", grad_weight)])
    g, et = _rgcn_cgraph(graph, etypes, norm, weight.shape[0], 1)
    check_call(_ffi.lib().DGLMIRgcnLayer1Backward(
        ctypes.byref(g), _arr(hidden, "hidden"), _arr(weight, "weight"), _arr(norm, "norm"),
        _arr(grad_out, "grad_out"), _arr(grad_hidden, "grad_hidden"),
        _arr(grad_weight, "grad_weight"), _stream(grad_out)))
