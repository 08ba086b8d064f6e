"""Graph index: edge storage plus the per-device CSR pair the kernels walk.

Restates the provisioning rules of the reference (``python/dgl/graph_index.py``
and ``src/graph/{graph,immutable_graph}.cc``):

* a mutable graph stores edges in insertion (edge-id) order;
* its out-CSR is the adjacency list in edge-id order (``graph.cc:600-660``),
  i.e. ``COOToCSR(src, dst)`` (a stable counting sort);
* its in-CSR is ``CSRTranspose(out-CSR)`` (``immutable_graph.cc:407-436``),
  so every destination row lists (src asc, eid asc);
* the immutable index is built lazily and cached per device
  (``graph_index.py:671-686``); any mutation drops the cache.

MI355X specifics: device CSRs are int32 (the reference GPU path is int32
only, ``kernel/common.h:62-69``) and carry the row id of every position
(``rows``), which the edge-wise and load-balanced kernels read.  A graph of 2^31
or more edges -- where the reference switches to int64 (``bits_needed``,
``graph_index.py:941-952``) and only its CPU kernels run -- gets 64-bit offsets:
int64 ``indptr`` and ``data`` (edge ids), int32 ``indices`` / ``rows`` (node ids
stay below 2^31; 288 GB of HBM holds such a graph, about 16 B per edge and
direction).  ``GraphIndex.asbits(64)`` forces that layout on any graph (parity
tests).  Large graphs can be built directly on the GPU
(:meth:`GraphIndex.from_device_coo`): stable radix sorts give arrays
bit-identical to the host path.
"""
from __future__ import annotations

import ctypes
import os

import weakref

import numpy as np
import torch as th

from . import _ffi
from ._ffi import DGLError


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class DeviceCSR:
    """One direction of the adjacency on a device: int32 arrays, or int64
    ``indptr`` / ``data`` for a 64-bit graph."""

    def __init__(self, indptr, indices, data, rows, num_cols):
        self.bits = 64 if indptr.dtype == th.int64 else 32
        self.indptr = indptr
        self.indices = indices
        self.data = data
        self.rows = rows
        self.num_rows = int(indptr.shape[0]) - 1
        self.num_cols = int(num_cols)
        self.nnz = int(indices.shape[0])

    def cstruct(self):
        """The C struct of this CSR (arrays are immutable: built once, then copied)."""
        if getattr(self, "_c", None) is None:
            self._c = self._make_cstruct()
        return _ffi.CSR.from_buffer_copy(self._c)

    def _make_cstruct(self):
        c = _ffi.CSR()
        c.num_rows = self.num_rows
        c.num_cols = self.num_cols
        c.nnz = self.nnz
        c.indptr = self.indptr.data_ptr()
        c.indices = self.indices.data_ptr() if self.nnz else None
        c.data = self.data.data_ptr() if self.nnz else None
        c.rows = self.rows.data_ptr() if self.nnz else None
        return c

    def degrees(self):
        """Row degrees on the device (the indptr's dtype), computed once and cached."""
        if getattr(self, "_deg", None) is None:
            self._deg = self.indptr[1:] - self.indptr[:-1]
        return self._deg


class ImmutableGraphIndex:
    """The kernels' view of a graph on one device: in-CSR + out-CSR."""

    def __init__(self, in_csr, out_csr, num_src, num_dst, device, eid_perm=False):
        self.in_csr = in_csr
        self.out_csr = out_csr
        self.num_src = num_src
        self.num_dst = num_dst
        self.device = device
        # in_csr.data is a permutation of [0, nnz) (whole graphs; parent-eid
        # subgraphs are not), so an edge-id ordered COO exists
        self.eid_perm = eid_perm
        self._coo = None
        self._gather_cols = None
        self._col_blocks = {}
        # "in" / "out" for a position view (position_view): edge ids = that walk's positions
        self.position_of = None
        # relation id per edge id (int32 on the device) for the R-GCN entries, which
        # read it from the graph like the reference (DGLMIGraph.etypes); None = untyped
        self.etypes = None

    def set_edge_types(self, etypes):
        """Attach the relation id of every edge (int32-convertible, one per edge id)."""
        if etypes is None:
            self.etypes = None
            return self
        t = th.as_tensor(etypes).reshape(-1)
        if t.numel() != self.in_csr.nnz:
            raise DGLError("etypes needs one entry per edge (%d, got %d)"
                           % (self.in_csr.nnz, t.numel()))
        if t.numel() and int(t.min()) < 0:
            raise DGLError("negative edge type")
        self.etypes = t.to(device=self.in_csr.indices.device, dtype=th.int32).contiguous()
        return self

    def number_of_edges(self):
        return self.in_csr.nnz

    @property
    def num_bits(self):
        """32, or 64 when indptr / edge ids are int64 (DGLMIGraph.num_bits)."""
        return self.in_csr.bits

    def coo(self):
        """(src, dst) by edge id, int32 on the device, scattered from the in-CSR
        once and cached (8 B per edge); None for parent-eid subgraphs."""
        if not self.eid_perm:
            return None
        if self._coo is None:
            c = self.in_csr
            src = th.empty(c.nnz, dtype=th.int32, device=c.indices.device)
            dst = th.empty_like(src)
            if c.nnz:
                e = c.data.long()
                src[e] = c.indices
                dst[e] = c.rows
            self._coo = (src, dst)
        return self._coo

    # Cold-row hints (DGLMIGraph.{in,out}_gather_cols): built for graphs whose node
    # tables can outgrow the 256 MiB Infinity Cache (>= 2^20 nodes on a side and
    # >= 2^22 edges); the library uses them only when the gathered table is
    # >= 256 MiB.  A row gathered fewer than HOT_DEGREE times per pass is cold.
    # M1 sweep (scripts/hotcold_probe.py, profiles/r01_hotcold_w{1,8}.json): the
    # hot set at degree >= 64 gives 3.24 -> 3.11 ms forward, 3.26 -> 3.12 ms
    # source gradient (world 1) and 3.69 -> 3.52 ms forward (a rank of world 8),
    # bit-identical; thresholds 16 / 32 / 128 / 256 are no better; every row
    # non-temporal: 5.5 ms.
    HOT_DEGREE = 64
    MAX_COLD_SHARE = 0.5
    MIN_HINT_NODES = 1 << 20
    MIN_HINT_EDGES = 1 << 22

    def gather_cols(self):
        """(in, out) cold-marked column arrays, built on the device once and cached
        (4 B per edge and direction); (None, None) for small graphs."""
        if self._gather_cols is None:
            self._gather_cols = (None, None)
            hot = int(os.environ.get("DGLMI_HOT_DEGREE", self.HOT_DEGREE))
            if hot > 0 and self.in_csr.nnz >= self.MIN_HINT_EDGES:
                cols = []
                g = self._cstruct_base()
                for direction, csr in ((0, self.in_csr), (1, self.out_csr)):
                    if csr.num_cols < self.MIN_HINT_NODES:
                        cols.append(None)
                        continue
                    out = th.empty(csr.nnz, dtype=th.int32, device=csr.indices.device)
                    _ffi.check_call(_ffi.lib().DGLMIKernelMarkColdColumns(
                        ctypes.byref(g), direction, hot, out.data_ptr(),
                        th.cuda.current_stream(csr.indices.device).cuda_stream))
                    # mostly-cold tables (no hot set worth protecting) gain nothing and
                    # lose a little: C5's typed graph, 4 edges per row, 3.82 -> 3.94 ms
                    if float((out < 0).float().mean()) > self.MAX_COLD_SHARE:
                        out = None
                    cols.append(out)
                self._gather_cols = tuple(cols)
        return self._gather_cols

    @staticmethod
    def _split_by_column(csr, nb):
        """``nb`` full-height CSRs holding csr's positions whose column lies in the
        b-th of nb equal id ranges, positions in their original order (a stable
        sort by block), built on the device."""
        dev = csr.indices.device
        n_rows = csr.num_rows
        key = (csr.indices.long() * nb) // max(1, csr.num_cols)
        order = th.argsort(key, stable=True)
        counts = th.bincount(key, minlength=nb).tolist()
        rows, cols, data = csr.rows[order], csr.indices[order], csr.data[order]
        del order, key
        out, start = [], 0
        for b in range(nb):
            end = start + counts[b]
            r = rows[start:end]
            indptr = th.zeros(n_rows + 1, dtype=th.int64, device=dev)
            indptr[1:] = th.cumsum(th.bincount(r.long(), minlength=n_rows), 0)
            out.append(DeviceCSR(indptr.to(th.int32), cols[start:end], data[start:end], r,
                                 csr.num_cols))
            start = end
        return out

    def position_operand(self, w, direction="in"):
        """(view, w_pos): a view of this graph whose edge ids are the positions of
        its in-CSR (``direction="in"``, for reductions to destinations) or of its
        out-CSR (``"out"``, for source-side gradients), and the per-edge operand
        ``w`` permuted into that order, so the walk streams it instead of
        gathering it by edge id (C5 typed gather 6.57 -> 5.60 ms, bit-identical;
        scripts/typed_probe.py).  For constant operands (R-GCN's norm): the
        permuted copy is cached per direction for the last (tensor, version)
        seen."""
        ic, oc = self.in_csr, self.out_csr
        view = self.position_view(direction)
        walk = ic if direction == "in" else oc
        # (address, version counter, layout) identifies `w`'s contents while `w` is
        # alive; the cache holds `w` only by a weak reference whose callback drops the
        # entry (and the permuted copy) the moment `w` is freed, so a dropped operand
        # costs no memory and its address cannot be mistaken for a later tensor's
        # The weak reference is to the STORAGE OWNER (``w._base`` for a view): a caller
        # that hands a fresh view of the same tensor each call (_typed_aggregate's
        # ``norm.reshape(E, 1)``) still hits, and the entry lives as long as the data.
        key = self._operand_key(w)
        owner = w._base if w._base is not None else w
        cached = self._pos_operands.get(direction)
        if cached is None or cached[0] != key or cached[1]() is not owner:
            ops = self._pos_operands

            def drop(ref, direction=direction):
                ent = ops.get(direction)
                if ent is not None and ent[1] is ref:
                    del ops[direction]
            from . import kernel as K
            cached = (key, weakref.ref(owner, drop), K.gather_rows(w, walk.data))
            self._pos_operands[direction] = cached
        return view, cached[2]

    def clear_operand_cache(self):
        """Drop the cached position-ordered operand copies (position_operand) and the
        last-seen operand record (reused_operand)."""
        if getattr(self, "_pos_operands", None) is not None:
            self._pos_operands.clear()
        self._operand_seen = None

    @staticmethod
    def _operand_key(w):
        return (w.data_ptr(), w._version, tuple(w.shape), tuple(w.stride()), w.dtype)

    def reused_operand(self, w):
        """True when ``w`` (same storage, version and layout) is the operand whose
        position-ordered copy is cached, or was seen by the previous call: a permuted
        copy pays off only for an operand used more than once (a fresh attention
        tensor per call would pay a full permutation each time)."""
        key = self._operand_key(w)
        if getattr(self, "_pos_views", None) is None:
            self._pos_views, self._pos_operands = {}, {}
        cached = self._pos_operands.get("in")
        owner = w._base if w._base is not None else w
        if cached is not None and cached[0] == key and cached[1]() is owner:
            return True
        # the same tensor OBJECT (a weak reference: the caching allocator hands a
        # fresh tensor of the same size the same address, so the key alone would
        # take each call's new attention tensor for the last one)
        prev = getattr(self, "_operand_seen", None)
        seen = prev is not None and prev[0]() is w and prev[1] == key
        self._operand_seen = (weakref.ref(w), key)
        return seen

    def position_view(self, direction):
        """This graph with edge ids = positions of its in-CSR (``"in"``) or out-CSR
        (``"out"``), so a per-edge operand in that walk's order is streamed."""
        ic, oc = self.in_csr, self.out_csr
        if getattr(self, "_pos_views", None) is None:
            self._pos_views, self._pos_operands = {}, {}
        if direction not in self._pos_views:
            dev = ic.indices.device
            pos = th.arange(ic.nnz, device=dev, dtype=ic.data.dtype)
            walk, other = (ic, oc) if direction == "in" else (oc, ic)
            inv = th.empty_like(pos)
            inv[walk.data.long()] = pos
            wv = DeviceCSR(walk.indptr, walk.indices, pos, walk.rows, walk.num_cols)
            ov = DeviceCSR(other.indptr, other.indices, inv[other.data.long()], other.rows,
                           other.num_cols)
            view = ImmutableGraphIndex(
                wv if direction == "in" else ov, ov if direction == "in" else wv,
                self.num_src, self.num_dst, self.device, eid_perm=True)
            view.position_of = direction  # its edge ids are this walk's positions
            self._pos_views[direction] = view
        return self._pos_views[direction]

    def gcn_edge_weights(self, norm):
        """GraphConv's normalisation as one constant weight per edge, in the walk
        order of each direction (built once, cached): ``"both"`` w = d_out(u)^-1/2 *
        d_in(v)^-1/2, ``"right"`` w = 1 / d_in(v) (degrees clamped at 1,
        graphconv.py:150-170).  Returns (in-view, w_in, out-view, w_out)."""
        cache = self.__dict__.setdefault("_gcn_w", {})
        if norm not in cache:
            ic, oc = self.in_csr, self.out_csr
            d_in = ic.degrees().float().clamp(min=1)
            d_out = oc.degrees().float().clamp(min=1)
            if norm == "both":
                ns, nd = th.pow(d_out, -0.5), th.pow(d_in, -0.5)
                w_in = ns[ic.indices.long()] * nd[ic.rows.long()]
                w_out = ns[oc.rows.long()] * nd[oc.indices.long()]
            else:
                nd = 1.0 / d_in
                w_in = nd[ic.rows.long()]
                w_out = nd[oc.indices.long()]
            cache[norm] = (self.position_view("in"), w_in.reshape(-1, 1).contiguous(),
                           self.position_view("out"), w_out.reshape(-1, 1).contiguous())
        return cache[norm]

    def col_blocks(self, nb):
        """(in_blocks, out_blocks): the in-CSR split by source range and the
        out-CSR by destination range into ``nb`` blocks each (DGLMIGraph
        .{in,out}_col_blocks), built once per ``nb`` and cached."""
        if nb not in self._col_blocks:
            self._col_blocks[nb] = (self._split_by_column(self.in_csr, nb),
                                    self._split_by_column(self.out_csr, nb))
        return self._col_blocks[nb]

    def _cstruct_base(self):
        g = _ffi.Graph()
        g.in_csr = self.in_csr.cstruct()
        g.out_csr = self.out_csr.cstruct()
        g.num_bits = self.num_bits
        g.device = self.device.index if self.device.index is not None else th.cuda.current_device()
        g.workspace = None
        g.workspace_bytes = 0
        return g

    def gat_edge_pos(self):
        """DGLMIGraph.gat_edge_pos: for every in-CSR position, the out-CSR position of
        the same edge, built once on the device (int32, 4 B per edge)."""
        if getattr(self, "_gat_pos", None) is None:
            ic, oc = self.in_csr, self.out_csr
            dev = ic.indices.device
            inv = th.empty(ic.nnz, dtype=th.int32, device=dev)
            inv[oc.data.long()] = th.arange(oc.nnz, dtype=th.int32, device=dev)
            self._gat_pos = inv[ic.data.long()].contiguous()
        return self._gat_pos

    def cstruct(self, workspace=None, coo=False, col_blocks=0, edge_pos=False):
        """The DGLMIGraph of a call: a cached template per (coo, col_blocks, edge_pos)
        -- every pointer in it is fixed for the graph's life -- copied, plus the call's
        workspace (cuts the host cost of a launch-bound call, C1-size graphs)."""
        if self.num_bits == 64:
            col_blocks, edge_pos = 0, False  # the blocked and GAT kernels are int32-only
        edge_pos = bool(edge_pos) and self.eid_perm and self.in_csr.nnz > 0 and col_blocks <= 1
        key = (bool(coo), int(col_blocks), edge_pos)
        tmpls = self.__dict__.setdefault("_ctmpl", {})
        if key not in tmpls:
            tmpls[key] = self._make_cstruct(coo, col_blocks)
            if edge_pos:
                tmpls[key].gat_edge_pos = self.gat_edge_pos().data_ptr()
        g = _ffi.Graph.from_buffer_copy(tmpls[key])
        if workspace is not None:
            g.workspace = workspace.data_ptr()
            g.workspace_bytes = workspace.numel() * workspace.element_size()
        return g

    def _make_cstruct(self, coo, col_blocks):
        g = _ffi.Graph()
        if col_blocks > 1:
            ib, ob = self.col_blocks(col_blocks)
            arr_i = (_ffi.CSR * col_blocks)(*[c.cstruct() for c in ib])
            arr_o = (_ffi.CSR * col_blocks)(*[c.cstruct() for c in ob])
            g._keep = (arr_i, arr_o)  # alive as long as the struct
            g.num_col_blocks = col_blocks
            g.in_col_blocks = ctypes.cast(arr_i, ctypes.c_void_p)
            g.out_col_blocks = ctypes.cast(arr_o, ctypes.c_void_p)
        g.in_csr = self.in_csr.cstruct()
        g.out_csr = self.out_csr.cstruct()
        pair = self.coo() if coo else None
        g.coo_src = pair[0].data_ptr() if pair is not None and self.in_csr.nnz else None
        g.coo_dst = pair[1].data_ptr() if pair is not None and self.in_csr.nnz else None
        ic, oc = self.gather_cols()
        g.in_gather_cols = ic.data_ptr() if ic is not None else None
        g.out_gather_cols = oc.data_ptr() if oc is not None else None
        g.num_bits = self.num_bits
        g.device = self.device.index if self.device.index is not None else th.cuda.current_device()
        g.workspace = None
        g.workspace_bytes = 0
        g.eid_identity = self.eid_identity_bits()
        return g

    def eid_identity_bits(self):
        """DGLMIGraph.eid_identity: bit 0 when the in-CSR's edge ids are its positions,
        bit 1 the same for the out-CSR -- a position view's walk, or a whole graph whose
        edges came sorted by destination (by source): its edge operands are then read
        at the walk position, streamed, instead of gathered by edge id.  Checked once
        on the device and cached (DGLMI_EID_IDENTITY=0 turns the detection off)."""
        if self.position_of is not None:
            return {"in": 1, "out": 2}[self.position_of]
        bits = getattr(self, "_eid_id_bits", None)
        if bits is None:
            bits = 0
            if self.eid_perm and self.in_csr.nnz and os.environ.get("DGLMI_EID_IDENTITY", "1") != "0":
                for bit, c in ((1, self.in_csr), (2, self.out_csr)):
                    iota = th.arange(c.nnz, device=c.data.device, dtype=c.data.dtype)
                    if bool(th.equal(c.data, iota)):
                        bits |= bit
                    del iota
            self._eid_id_bits = bits
        return bits

    def workspace_bytes(self, feat_len):
        cache = self.__dict__.setdefault("_ws_bytes", {})
        if feat_len not in cache:
            L = _ffi.lib()
            a = L.DGLMIKernelWorkspaceBytes(ctypes.byref(self.in_csr.cstruct()), int(feat_len))
            b = L.DGLMIKernelWorkspaceBytes(ctypes.byref(self.out_csr.cstruct()), int(feat_len))
            cache[feat_len] = max(a, b)
        return cache[feat_len]


def host_coo_to_csr(num_rows, row, col, data=None):
    """aten::COOToCSR through the C ABI (int64 host arrays)."""
    row = np.ascontiguousarray(row, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int64)
    data = None if data is None else np.ascontiguousarray(data, dtype=np.int64)
    nnz = row.shape[0]
    indptr = np.empty(num_rows + 1, np.int64)
    indices = np.empty(nnz, np.int64)
    out = np.empty(nnz, np.int64)
    _p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
    rc = _ffi.lib().DGLMICOOToCSR(num_rows, nnz, _p(row), _p(col), _p(data), _p(indptr),
                                  _p(indices), _p(out))
    if rc != 0:
        raise DGLError("COOToCSR: row id out of range")
    return indptr, indices, out


def host_csr_transpose(num_rows, num_cols, indptr, indices, data=None):
    """aten::CSRTranspose through the C ABI (int64 host arrays)."""
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int64)
    data = None if data is None else np.ascontiguousarray(data, dtype=np.int64)
    nnz = indices.shape[0]
    bp = np.empty(num_cols + 1, np.int64)
    bi = np.empty(nnz, np.int64)
    bx = np.empty(nnz, np.int64)
    _p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
    rc = _ffi.lib().DGLMICSRTranspose(num_rows, num_cols, _p(indptr), _p(indices), _p(data),
                                      _p(bp), _p(bi), _p(bx))
    if rc != 0:
        raise DGLError("CSRTranspose: column id out of range")
    return bp, bi, bx


def _stream_ptr(device):
    return ctypes.c_void_p(th.cuda.current_stream(device).cuda_stream)


def device_coo_to_csr(num_rows, row, col, data=None):
    """COO -> CSR on the GPU (int32 tensors), bit-identical to host_coo_to_csr."""
    dev = row.device
    nnz = int(row.shape[0])
    L = _ffi.lib()
    indptr = th.empty(num_rows + 1, dtype=th.int32, device=dev)
    indices = th.empty(nnz, dtype=th.int32, device=dev)
    out = th.empty(nnz, dtype=th.int32, device=dev)
    ws = th.empty(int(L.DGLMICOOToCSRDeviceWorkspaceBytes(num_rows, nnz)), dtype=th.uint8, device=dev)
    rc = L.DGLMICOOToCSRDevice(num_rows, nnz, _ptr(row), _ptr(col), _ptr(data), _ptr(indptr),
                               _ptr(indices), _ptr(out), _ptr(ws), ws.numel(), _stream_ptr(dev))
    if rc != 0:
        raise DGLError("device COOToCSR failed")
    return indptr, indices, out


def device_expand_rows(indptr, nnz):
    rows = th.empty(nnz, dtype=th.int32, device=indptr.device)
    if nnz:
        fn = (_ffi.lib().DGLMICSRExpandRows64 if indptr.dtype == th.int64
              else _ffi.lib().DGLMICSRExpandRows)
        rc = fn(_ptr(indptr), indptr.shape[0] - 1, nnz, _ptr(rows), _stream_ptr(indptr.device))
        if rc != 0:
            raise DGLError("CSR row expansion failed")
    return rows


def device_coo_to_csr64(num_rows, row, col, data=None):
    """COO -> CSR on the GPU for 64-bit graphs: int32 row / col, optional int64 data;
    returns int64 indptr, int32 indices, int64 data (edge ids), bit-identical to
    host_coo_to_csr."""
    dev = row.device
    nnz = int(row.shape[0])
    L = _ffi.lib()
    indptr = th.empty(num_rows + 1, dtype=th.int64, device=dev)
    indices = th.empty(nnz, dtype=th.int32, device=dev)
    out = th.empty(nnz, dtype=th.int64, device=dev)
    ws = th.empty(int(L.DGLMICOOToCSRDevice64WorkspaceBytes(num_rows, nnz)), dtype=th.uint8,
                  device=dev)
    rc = L.DGLMICOOToCSRDevice64(num_rows, nnz, _ptr(row), _ptr(col), _ptr(data), _ptr(indptr),
                                 _ptr(indices), _ptr(out), _ptr(ws), ws.numel(), _stream_ptr(dev))
    if rc != 0:
        raise DGLError("device COOToCSR (64-bit) failed")
    return indptr, indices, out


MAX_NODES = 0x7FFFFFFF  # node ids are int32 on the device, in both layouts


def device_block_gidx(num_src, num_dst, src, dst, bits=None):
    """In/out CSRs of a (num_src -> num_dst) block from device int32 COO, on the GPU.

    out-CSR = stable sort of the eid-ordered COO by src; in-CSR = stable re-sort
    of that sequence by dst == CSRTranspose(out-CSR) (``spmat_op_impl.cc:323-369``),
    so every dst row lists its sources ascending, eids ascending within a source.
    """
    dev = src.device
    m = int(src.shape[0])
    if max(int(num_src), int(num_dst)) >= MAX_NODES:
        raise DGLError("Unsupported graph: 2^31 or more nodes (device node ids are int32)")
    if bits is None:
        bits = 64 if m >= 0x7FFFFFFF else 32
    src = src.to(th.int32).contiguous()
    dst = dst.to(th.int32).contiguous()
    build = device_coo_to_csr64 if bits == 64 else device_coo_to_csr
    o_ptr, o_idx, o_dat = build(num_src, src, dst)
    o_rows = device_expand_rows(o_ptr, m)
    i_ptr, i_idx, i_dat = build(num_dst, o_idx, o_rows, o_dat)
    i_rows = device_expand_rows(i_ptr, m)
    return ImmutableGraphIndex(DeviceCSR(i_ptr, i_idx, i_dat, i_rows, num_src),
                               DeviceCSR(o_ptr, o_idx, o_dat, o_rows, num_dst),
                               num_src, num_dst, dev, eid_perm=True)


class GraphIndex:
    """Mutable multigraph index (``python/dgl/graph_index.py:GraphIndex``)."""
    _eid_is_perm = True  # CSR data = own edge ids 0..E-1 (subgraph views override)

    def __init__(self, num_nodes=0):
        self._n = int(num_nodes)
        self._src = np.empty(0, np.int64)
        self._dst = np.empty(0, np.int64)
        self._cache = {}
        self._host_csr = None
        self._degs = None
        self._etype = None        # per-edge relation ids (add_edges_with_type), numpy int64
        self._typed = {}
        self._device_only = None  # (src, dst) device tensors when built on the GPU
        self._bits = None         # forced device index width (asbits)

    # ---- construction -----------------------------------------------------
    @classmethod
    def from_device_coo(cls, src, dst, num_nodes):
        """Build directly from device int32 (src, dst) tensors (no host copy)."""
        g = cls(num_nodes)
        g._device_only = (src, dst)
        g._m = int(src.shape[0])
        return g

    def _invalidate(self):
        self._cache = {}
        self._host_csr = None
        self._degs = None
        self._typed = {}

    def add_nodes(self, num):
        if self._device_only is not None:
            raise DGLError("graph built on device is immutable")
        self._n += int(num)
        self._invalidate()

    def add_edges_with_type(self, u, v, etypes):
        """graph.py:1229 (hack): edges plus their relation ids."""
        old = self.number_of_edges()
        self.add_edges(u, v)
        t = np.atleast_1d(np.asarray(etypes, dtype=np.int64))
        m = self.number_of_edges() - old
        if t.shape[0] == 1 and m > 1:
            t = np.full(m, t[0], np.int64)
        if t.shape[0] != m:
            raise DGLError("etypes length %d != number of new edges %d" % (t.shape[0], m))
        prev = self._etype if self._etype is not None else np.zeros(old, np.int64)
        self._etype = np.concatenate([prev, t])

    def edge_types(self):
        if self._etype is None:
            return None
        if self._etype.shape[0] != self.number_of_edges():  # untyped edges added later
            pad = np.zeros(self.number_of_edges() - self._etype.shape[0], np.int64)
            self._etype = np.concatenate([self._etype, pad])
        return self._etype

    def typed_gidx(self, device, num_rels, etypes=None, node_major=False):
        """Relation-expanded graph for R-GCN: source (type_e * N + u) -> v, R*N sources
        (relation-major rows, as a (R, N, F) weight/feature tensor is laid out), or
        source (u * R + type_e) with ``node_major`` (the rows of one (N, R*F) GEMM
        output X @ [W_0 | ... | W_{R-1}]).

        Built on the device (two stable radix sorts) and cached per (device, R, etypes, layout)."""
        device = th.device(device)
        if etypes is None:
            et = self.edge_types()
            if et is None:
                raise DGLError("graph has no edge types; pass etypes")
            key = (str(device), int(num_rels), "graph", bool(node_major))
            etypes = th.from_numpy(et)
        else:
            key = (str(device), int(num_rels), etypes.data_ptr(), etypes._version,
                   int(etypes.shape[0]), bool(node_major))
        if key not in self._typed:
            n = self._n
            if num_rels * n >= 0x7FFFFFFF:
                raise DGLError("num_rels * num_nodes exceeds int32 indexing")
            if self._device_only is not None:
                src, dst = (t.to(device=device, dtype=th.int64) for t in self._device_only)
            else:
                src = th.from_numpy(self._src).to(device)
                dst = th.from_numpy(self._dst).to(device)
            et = etypes.to(device=device, dtype=th.int64).reshape(-1)
            if et.shape[0] != src.shape[0]:
                raise DGLError("etypes must have one entry per edge")
            if et.numel() and (int(et.min()) < 0 or int(et.max()) >= num_rels):
                raise DGLError("edge type out of range [0, %d)" % num_rels)
            tsrc = ((src * num_rels + et) if node_major else (et * n + src)).to(th.int32).contiguous()
            self._typed[key] = device_block_gidx(num_rels * n, n, tsrc, dst)
        return self._typed[key]

    def add_edges(self, u, v):
        if self._device_only is not None:
            raise DGLError("graph built on device is immutable")
        u = np.atleast_1d(np.asarray(u, dtype=np.int64))
        v = np.atleast_1d(np.asarray(v, dtype=np.int64))
        if u.shape[0] == 1 and v.shape[0] > 1:
            u = np.full(v.shape, u[0], np.int64)
        if v.shape[0] == 1 and u.shape[0] > 1:
            v = np.full(u.shape, v[0], np.int64)
        if u.shape != v.shape:
            raise DGLError("Invalid src/dst lengths: %d vs %d" % (u.shape[0], v.shape[0]))
        if u.size and (u.min() < 0 or v.min() < 0 or u.max() >= self._n or v.max() >= self._n):
            raise DGLError("Invalid node id in add_edges (graph has %d nodes)" % self._n)
        self._src = np.concatenate([self._src, u])
        self._dst = np.concatenate([self._dst, v])
        self._invalidate()

    # ---- queries ----------------------------------------------------------
    def number_of_nodes(self):
        return self._n

    def number_of_edges(self):
        if self._device_only is not None:
            return self._m
        return int(self._src.shape[0])

    def bits_needed(self):
        # graph_index.py:941-952
        return 32 if max(self._n, self.number_of_edges()) < 0x7FFFFFFF else 64

    def device_bits(self):
        """Index width of the device CSRs: bits_needed(), or 64 when forced by asbits."""
        return 64 if self._bits == 64 else self.bits_needed()

    def asbits(self, bits):
        """graph_index.py:954-967: the same graph with the given index width.  Here
        the device CSRs of the returned index use int64 offsets and edge ids when
        ``bits`` is 64 (any graph, so small graphs exercise the 64-bit kernels);
        32 keeps the width bits_needed() asks for."""
        if bits not in (32, 64):
            raise DGLError("Invalid bit width: %s (32 or 64)" % bits)
        g = self.__class__.__new__(self.__class__)
        g.__dict__.update(self.__dict__)
        g._cache, g._typed = {}, {}
        g._bits = bits if bits == 64 else None
        return g

    def edges(self):
        """(src, dst, eid) in edge-id order (numpy int64)."""
        if self._device_only is not None:
            s, d = self._device_only
            return (s.long().cpu().numpy(), d.long().cpu().numpy(), np.arange(self._m))
        return self._src, self._dst, np.arange(self._src.shape[0], dtype=np.int64)

    def _degrees(self):
        """(in, out) degrees, cached; device-built graphs read them off their CSRs."""
        if self._degs is None:
            if self._device_only is not None:
                g = self.get_immutable_gidx(self._device_only[0].device)
                self._degs = (g.in_csr.degrees().long().cpu().numpy(),
                              g.out_csr.degrees().long().cpu().numpy())
            else:
                src, dst, _ = self.edges()
                self._degs = (np.bincount(dst, minlength=self._n).astype(np.int64),
                              np.bincount(src, minlength=self._n).astype(np.int64))
        return self._degs

    def in_degrees(self):
        return self._degrees()[0]

    def out_degrees(self):
        return self._degrees()[1]

    def host_csr(self):
        """(out-CSR, in-CSR) host arrays, int64, bit-exact with the reference."""
        if self._host_csr is None:
            src, dst, _ = self.edges()
            out_csr = host_coo_to_csr(self._n, src, dst)
            in_csr = host_csr_transpose(self._n, self._n, *out_csr)
            self._host_csr = (out_csr, in_csr)
        return self._host_csr

    def get_immutable_gidx(self, device):
        """The per-device CSR pair, built once and cached (graph_index.py:671-686)."""
        device = th.device(device)
        if device.type != "cuda":
            raise DGLError("the MI355X engine runs on ROCm devices only; got device %s" % device)
        if device.index is None:
            device = th.device("cuda", th.cuda.current_device())
        key = str(device)
        if key not in self._cache:
            if self._n >= MAX_NODES:
                raise DGLError("Unsupported graph: 2^31 or more nodes (device node ids are int32)")
            if self._device_only is not None:
                self._cache[key] = self._build_on_device(device)
            else:
                self._cache[key] = self._upload(device)
            self._cache[key].eid_perm = self._eid_is_perm
            et = self.edge_types() if self._eid_is_perm else None
            if et is not None:  # add_edges_with_type: the graph carries its relations
                self._cache[key].set_edge_types(th.from_numpy(et))
        return self._cache[key]

    def _upload(self, device):
        (op, oi, od), (ip, ii, idd) = self.host_csr()
        n = self._n
        off = np.int64 if self.device_bits() == 64 else np.int32

        def mk(indptr, indices, data):
            rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(indptr).astype(np.int64))
            t = lambda a, dt=np.int32: th.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(device)
            return DeviceCSR(t(indptr, off), t(indices), t(data, off), t(rows), n)

        return ImmutableGraphIndex(mk(ip, ii, idd), mk(op, oi, od), n, n, device)

    def _build_on_device(self, device):
        src, dst = self._device_only
        g = device_block_gidx(self._n, self._n, src.to(device), dst.to(device),
                              bits=self.device_bits())
        g.device = th.device(device)
        return g
