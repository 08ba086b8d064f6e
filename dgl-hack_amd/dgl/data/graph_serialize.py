"""Graph files in the reference's binary format (``python/dgl/data/graph_serialize.py:63-160``,
``src/graph/graph_serialize.cc:130-301``).

A file of int / uint / float tensors written here loads in the reference and the other
way round.  bool and bfloat16 tensors are written with DLPack codes 6 and 4, which
this library reads back; the reference's dlpack submodule is absent from its tree and
older DLPack releases define only Int / UInt / Float, so whether the reference loads
them is parity unpinned (convert to uint8 / float32 for a file the reference must
read).  Layout (little-endian,
dmlc-core stream encoding -- ``third_party/dmlc-core`` ``include/dmlc/serializer.h``, a
submodule absent from the reference tree: a POD is its raw bytes, a ``std::string`` and a
``std::vector`` a ``uint64`` length followed by the elements, a ``std::pair`` its two halves):

* bytes 0..23: ``kDGLSerializeMagic``, then two ``uint64`` the writer emits as
  (version 1, graph type 1 = immutable) and the reader reads as (graph type, version)
  (``graph_serialize.cc:134-137`` / ``:186-194``; both are 1, so the order is moot);
  zeros up to byte 4096;
* ``uint64 num_graph``; ``vector<uint64> graph_indices`` (file offset of each graph);
  ``vector<int64> nodes_num_list``; ``vector<int64> edges_num_list``;
  ``vector<pair<string, NDArray>> labels`` (``:143-164``);
* per graph (``GraphDataObject::Save``, ``:247-255``): the in-CSR ``indptr``, ``indices``,
  ``edge_ids`` as NDArrays, then the node tensors and the edge tensors as
  ``vector<pair<string, NDArray>>``;
* an NDArray (``include/dgl/runtime/ndarray.h:408-457``): ``uint64 kDGLNDArrayMagic``,
  ``uint64 reserved``, ``DLContext`` {int32 device_type = 1 (CPU), int32 device_id = 0},
  ``int32 ndim``, ``DLDataType`` {uint8 code, uint8 bits, uint16 lanes}, ``int64 shape[ndim]``,
  ``int64 data_byte_size``, the data.

The in-CSR is the one ``ImmutableGraph::GetInCSR`` builds for a COO-born graph
(``immutable_graph.cc:407-420``: transpose the COO, ``COOToCSR``), here through the C ABI's
``DGLMICOOToCSR`` (``dglmi.h``), so within a destination row the edges keep edge-id order.
Loaded graphs are read-only, features come back as CPU tensors, as in the reference.
"""
import os
import struct

import numpy as np
import torch as th

from .._ffi import DGLError
from ..graph import DGLGraph
from ..graph_index import GraphIndex, host_coo_to_csr

__all__ = ["save_graphs", "load_graphs", "load_labels"]

_FILE_MAGIC = 0xDD2E4FF046B4A13F      # graph_serialize.cc:128
_ARRAY_MAGIC = 0xDD5E40F096B4A13F     # ndarray.h:408
_VERSION = 1
_IMMUTABLE = 1
_HEADER = 4096

# DLDataType codes: kDLInt 0, kDLUInt 1, kDLFloat 2, kDLBfloat 4, kDLBool 6 (dlpack.h)
_TORCH_TO_DL = {
    th.int8: (0, 8), th.int16: (0, 16), th.int32: (0, 32), th.int64: (0, 64),
    th.uint8: (1, 8), th.float16: (2, 16), th.float32: (2, 32), th.float64: (2, 64),
    th.bfloat16: (4, 16), th.bool: (6, 8),
}
_DL_TO_TORCH = {v: k for k, v in _TORCH_TO_DL.items()}


# ---- writer -------------------------------------------------------------------------
def _w_u64(fh, v):
    fh.write(struct.pack("<Q", v))


def _w_array(fh, t):
    """NDArray::Save (ndarray.h:410-457); device tensors are written as CPU arrays."""
    t = th.as_tensor(t).detach()
    if t.dtype not in _TORCH_TO_DL:
        raise DGLError("save_graphs: unsupported tensor dtype %s" % t.dtype)
    code, bits = _TORCH_TO_DL[t.dtype]
    t = t.to("cpu").contiguous()
    fh.write(struct.pack("<QQiii", _ARRAY_MAGIC, 0, 1, 0, t.dim()))
    fh.write(struct.pack("<BBH", code, bits, 1))
    fh.write(struct.pack("<%dq" % t.dim(), *t.shape))
    nbytes = t.numel() * t.element_size()
    fh.write(struct.pack("<q", nbytes))
    if nbytes:
        fh.write(t.view(th.uint8).numpy().tobytes() if t.dtype in (th.bfloat16, th.bool)
                 else t.numpy().tobytes())


def _w_named(fh, items):
    """vector<pair<string, NDArray>>."""
    items = list(items)
    _w_u64(fh, len(items))
    for name, t in items:
        b = str(name).encode("utf-8")
        _w_u64(fh, len(b))
        fh.write(b)
        _w_array(fh, t)


def _w_vec(fh, values, fmt):
    _w_u64(fh, len(values))
    if len(values):
        fh.write(struct.pack("<%d%s" % (len(values), fmt), *values))


def _in_csr(g):
    """(indptr, indices, edge_ids) of the graph's in-CSR, int64 (immutable_graph.cc:416)."""
    src, dst, _ = g._graph.edges()
    return host_coo_to_csr(g.number_of_nodes(), dst, src)


def save_graphs(filename, g_list, labels=None):
    """Save graphs, their node/edge features and graph labels (``graph_serialize.py:63-103``)."""
    if isinstance(g_list, DGLGraph):
        g_list = [g_list]
    for g in g_list:
        if not isinstance(g, DGLGraph):
            raise DGLError("save_graphs expects DGLGraph objects, got %s" % type(g))
    labels = {} if labels is None else dict(labels)
    n = len(g_list)
    with open(filename, "wb") as fh:
        fh.write(struct.pack("<QQQ", _FILE_MAGIC, _VERSION, _IMMUTABLE))
        fh.write(b"\0" * (_HEADER - 24))
        _w_u64(fh, n)
        at_indices = fh.tell()
        _w_vec(fh, [0] * n, "Q")
        _w_vec(fh, [g.number_of_nodes() for g in g_list], "q")
        _w_vec(fh, [g.number_of_edges() for g in g_list], "q")
        _w_named(fh, labels.items())
        offsets = []
        for g in g_list:
            offsets.append(fh.tell())
            indptr, indices, eids = _in_csr(g)
            for a in (indptr, indices, eids):
                _w_array(fh, th.from_numpy(a))
            _w_named(fh, g.ndata.items())
            _w_named(fh, g.edata.items())
        fh.seek(at_indices)
        _w_vec(fh, offsets, "Q")


# ---- reader -------------------------------------------------------------------------
class _Reader:
    def __init__(self, fh, size):
        self.fh = fh
        self.size = size

    def raw(self, n):
        b = self.fh.read(n)
        if len(b) != n:
            raise DGLError("Invalid DGL file: truncated")
        return b

    def u64(self):
        return struct.unpack("<Q", self.raw(8))[0]

    def vec(self, fmt, width):
        n = self.u64()
        if n * width > self.size:
            raise DGLError("Invalid DGL file: vector length %d" % n)
        return list(struct.unpack("<%d%s" % (n, fmt), self.raw(n * width))) if n else []

    def array(self):
        """NDArray::Load (ndarray.h:463-510)."""
        magic, _reserved, dev_type, _dev_id, ndim = struct.unpack("<QQiii", self.raw(28))
        if magic != _ARRAY_MAGIC:
            raise DGLError("Invalid DLTensor file format")
        if dev_type != 1:
            raise DGLError("Invalid DLTensor context: can only save as CPU tensor")
        code, bits, lanes = struct.unpack("<BBH", self.raw(4))
        if ndim < 0 or lanes != 1 or (code, bits) not in _DL_TO_TORCH:
            raise DGLError("Invalid DLTensor file format: dtype (%d, %d, %d)" % (code, bits, lanes))
        shape = struct.unpack("<%dq" % ndim, self.raw(8 * ndim)) if ndim else ()
        nbytes = struct.unpack("<q", self.raw(8))[0]
        dtype = _DL_TO_TORCH[(code, bits)]
        numel = int(np.prod(shape, dtype=np.int64)) if ndim else 1
        if nbytes != numel * (bits // 8):
            raise DGLError("Invalid DLTensor file format")
        buf = bytearray(self.raw(nbytes))
        t = th.frombuffer(buf, dtype=th.uint8) if nbytes else th.empty(0, dtype=th.uint8)
        return t.view(dtype).reshape(shape)

    def named(self):
        out = {}
        for _ in range(self.u64()):
            ln = self.u64()
            if ln > self.size:
                raise DGLError("Invalid DGL file: string length %d" % ln)
            name = self.raw(ln).decode("utf-8")
            out[name] = self.array()
        return out


def _read_meta(fh):
    size = os.fstat(fh.fileno()).st_size
    r = _Reader(fh, size)
    magic, gtype, version = struct.unpack("<QQQ", r.raw(24))
    if magic != _FILE_MAGIC:
        raise DGLError("Invalid DGL files")
    if gtype != _IMMUTABLE:
        raise DGLError("Invalid DGL files")
    if version != _VERSION:
        raise DGLError("Invalid Serialization Version")
    fh.seek(_HEADER)
    num_graph = r.u64()
    indices = r.vec("Q", 8)
    nodes = r.vec("q", 8)
    edges = r.vec("q", 8)
    labels = r.named()
    if not (len(indices) == len(nodes) == len(edges) == num_graph):
        raise DGLError("Invalid DGL file: graph tables disagree")
    return r, indices, nodes, edges, labels


def _read_graph(r):
    """GraphDataObject::Load (graph_serialize.cc:257-268): ImmutableGraph::CreateFromCSR(
    indptr, indices, edge_ids, "in") -- edge edge_ids[p] runs indices[p] -> row(p)."""
    indptr, indices, eids = (r.array().to(th.int64).numpy() for _ in range(3))
    n = indptr.shape[0] - 1
    m = indices.shape[0]
    if n < 0 or eids.shape[0] != m or indptr[0] != 0 or indptr[-1] != m or \
            np.any(np.diff(indptr) < 0):
        raise DGLError("Invalid DGL file: malformed in-CSR")
    if m and (indices.min() < 0 or indices.max() >= n or
              not np.array_equal(np.sort(eids), np.arange(m))):
        raise DGLError("Invalid DGL file: malformed in-CSR")
    src = np.empty(m, np.int64)
    dst = np.empty(m, np.int64)
    src[eids] = indices
    dst[eids] = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    gi = GraphIndex(n)
    gi.add_edges(src, dst)
    g = DGLGraph(gi, readonly=True)
    for k, v in r.named().items():
        g.ndata[k] = v
    for k, v in r.named().items():
        g.edata[k] = v
    return g


def load_graphs(filename, idx_list=None):
    """(graph list, label dict) from a file (``graph_serialize.py:106-139``); ``idx_list``
    selects graphs and orders the result."""
    if idx_list is None:
        idx_list = []
    if not isinstance(idx_list, list):
        raise DGLError("idx_list must be a list")
    with open(filename, "rb") as fh:
        r, offsets, _, _, labels = _read_meta(fh)
        if not idx_list:
            graphs = [_read_graph(r) for _ in offsets]
        else:
            graphs = []
            for i in idx_list:
                if not 0 <= int(i) < len(offsets):
                    raise DGLError("graph index %d out of range [0, %d)" % (i, len(offsets)))
                fh.seek(offsets[int(i)])
                graphs.append(_read_graph(r))
    return graphs, labels


def load_labels(filename):
    """The label dict alone (``graph_serialize.py:142-160``)."""
    with open(filename, "rb") as fh:
        return _read_meta(fh)[4]
