"""Host-side logic of the product (no GPU): C ABI exports, shape inference,
host graph ingestion, graph bookkeeping and error behaviour."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch as th

import dgl
import dgl.function as fn
from dgl import _ffi
from dgl.graph_index import GraphIndex, host_coo_to_csr, host_csr_transpose
from oracle import oracle as O
from graphs import er_graph, g20, powerlaw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = json.load(open(os.path.join(ROOT, "tests", "golden", "spmat_kat.json")))


def test_library_exports_header_symbols():
    hdr = open(os.path.join(ROOT, "include", "dglmi.h")).read()
    declared = set(re.findall(r"\b(DGLMI[A-Za-z0-9]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    lib = ctypes.CDLL(_ffi._lib_path())
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(_ffi.EXPORTED)
    assert _ffi.lib().DGLMIVersion() == b"0.4-mi355x"


@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "dot"])
def test_infer_shape_matches_oracle(op):
    rng = np.random.default_rng(0)
    shapes = [((7, 5, 3, 4), (9, 3, 1)), ((7, 4), (9, 5, 3, 4)), ((7, 5, 1, 4), (9, 5, 3, 4)),
              ((7, 1), (9, 6)), ((7, 2, 3), (9, 2, 3))]
    for a, b in shapes:
        if op == "dot" and a[-1] != b[-1]:
            continue
        x, y = th.zeros(a), th.zeros(b)
        assert dgl.kernel.infer_binary_feature_shape(op, x, y) == \
            O.infer_binary_feature_shape(op, x.numpy(), y.numpy())


def test_infer_shape_error():
    with pytest.raises(dgl.DGLError, match="Invalid broadcasting"):
        dgl.kernel.infer_binary_feature_shape("add", th.zeros(3, 5), th.zeros(3, 4))


def test_host_ingest_kat():
    for coo, csr in (("COO1", "CSR1"), ("COO2", "CSR2")):
        p, i, d = host_coo_to_csr(4, KAT[coo]["row"], KAT[coo]["col"])
        assert p.tolist() == KAT[csr]["indptr"]
        assert i.tolist() == KAT[csr]["indices"]
        assert d.tolist() == KAT[csr]["data"]
    c = KAT["CSR2"]
    p, i, d = host_csr_transpose(4, 5, c["indptr"], c["indices"], c["data"])
    assert p.tolist() == KAT["CSR2_T"]["indptr"]
    assert i.tolist() == KAT["CSR2_T"]["indices"]
    assert d.tolist() == KAT["CSR2_T"]["data"]


@pytest.mark.parametrize("maker", [g20, er_graph, lambda: powerlaw(5000, 60000, seed=2)])
def test_graph_csr_matches_oracle(maker):
    src, dst, n = maker()
    gi = GraphIndex(n)
    gi.add_edges(src, dst)
    (op, oi, od), (ip, ii, idd) = gi.host_csr()
    ref = O.RefGraph(src, dst, n)
    for a, b in zip((op, oi, od, ip, ii, idd), ref.out_csr + ref.in_csr):
        np.testing.assert_array_equal(a, b)


def test_ingest_rejects_bad_ids():
    with pytest.raises(dgl.DGLError):
        host_coo_to_csr(2, [0, 5], [0, 1])


def test_dglgraph_bookkeeping():
    g = dgl.DGLGraph()
    g.add_nodes(4)
    g.add_edges([0, 1, 2], [1, 2, 3])
    g.add_edge(3, 0)
    assert g.number_of_nodes() == 4 and g.number_of_edges() == 4
    assert g.in_degrees().tolist() == [1, 1, 1, 1]
    s, d = g.edges()
    assert s.tolist() == [0, 1, 2, 3] and d.tolist() == [1, 2, 3, 0]
    g.ndata["h"] = th.ones(4, 2)
    lv = g.local_var()
    lv.ndata["x"] = th.zeros(4, 1)
    assert "x" not in g.ndata and "h" in lv.ndata
    with pytest.raises(dgl.DGLError):
        g.ndata["bad"] = th.ones(3, 2)
    g.add_nodes(1)
    assert g.ndata["h"].shape == (5, 2)


def test_networkx_and_scipy_construction():
    import networkx as nx
    import scipy.sparse as sp
    g = dgl.DGLGraph(nx.path_graph(3))
    assert g.number_of_edges() == 4
    m = sp.coo_matrix((np.ones(3), ([0, 1, 2], [1, 2, 0])), shape=(3, 3))
    g2 = dgl.DGLGraph(m)
    assert g2.edges()[0].tolist() == [0, 1, 2]


def test_cpu_tensors_fail_loudly():
    g = dgl.DGLGraph()
    g.add_nodes(3)
    g.add_edges([0, 1], [1, 2])
    g.ndata["h"] = th.ones(3, 4)
    with pytest.raises(dgl.DGLError, match="ROCm"):
        g.update_all(fn.copy_u("h", "m"), fn.sum("m", "s"))


def test_udf_reduce_still_runs_builtin_messages_on_device():
    """A reduce UDF (degree bucketing) materialises builtin messages with the HIP
    kernel first: CPU tensors fail loudly there, no CPU fallback."""
    g = dgl.DGLGraph()
    g.add_nodes(2)
    g.add_edges([0], [1])
    g.ndata["h"] = th.zeros(2, 4)
    with pytest.raises(dgl.DGLError):
        g.update_all(fn.copy_u("h", "m"), lambda nodes: {"o": nodes.mailbox["m"].sum(1)})
    with pytest.raises(dgl.DGLError):  # a list must hold builtins only
        g.update_all(fn.copy_u("h", "m"), [fn.sum("m", "o"), lambda nodes: {}])


def test_capi_errors_without_device():
    """Reducer / op validation happens before any device work (binary_reduce_impl.h:95-98)."""
    L = _ffi.lib()
    g = _ffi.Graph()
    g.num_bits = 32
    a = _ffi.Array()
    rc = L.DGLMIKernelCopyReduce(b"mean", ctypes.byref(g), 0, ctypes.byref(a), ctypes.byref(a),
                                 None, None, None)
    assert rc == -1 and "reduce mean is not supported" in _ffi.last_error()
    rc = L.DGLMIKernelBinaryOpReduce(b"sum", b"pow", ctypes.byref(g), 0, 2, ctypes.byref(a),
                                     ctypes.byref(a), ctypes.byref(a), None, None, None, None)
    assert rc == -1 and "Unsupported binary op" in _ffi.last_error()
    g.num_bits = 16
    rc = L.DGLMIKernelCopyReduce(b"sum", ctypes.byref(g), 0, ctypes.byref(a), ctypes.byref(a),
                                 None, None, None)
    assert rc == -1 and "idx bits" in _ffi.last_error()
    # 64-bit graphs: mappings, and the int32-only entries, are refused before any device work
    g.num_bits = 64
    m = (ctypes.c_int32 * 2)()
    rc = L.DGLMIKernelCopyReduce(b"sum", ctypes.byref(g), 0, ctypes.byref(a), ctypes.byref(a),
                                 m, None, None)
    assert rc == -1 and "mappings need a graph of fewer than 2^31 edges" in _ffi.last_error()
    rc = L.DGLMIFusedGatForward(ctypes.byref(g), ctypes.byref(a), ctypes.byref(a), ctypes.byref(a),
                                0.2, ctypes.byref(a), ctypes.byref(a), ctypes.byref(a), None)
    assert rc == -1 and "fused GAT needs a graph of fewer than 2^31 edges" in _ffi.last_error()
    st = _ffi.RgcnState()
    rc = L.DGLMIRgcnPrepare(ctypes.byref(g), None, 2, 1, ctypes.byref(st), None)
    assert rc == -1 and "R-GCN needs a graph of fewer than 2^31 edges" in _ffi.last_error()


def test_builtin_names():
    assert fn.copy_src("a", "b").name == "copy_u"
    assert fn.copy_edge("a", "b").name == "copy_e"
    assert fn.src_mul_edge("a", "b", "c").name == "u_mul_e"
    assert fn.e_dot_v("a", "b", "c").name == "e_dot_v"
    assert fn.mean("m", "h").name == "mean"
    for lhs in "uve":
        for rhs in "uve":
            if lhs != rhs:
                for op in ["add", "sub", "mul", "div", "dot"]:
                    assert hasattr(fn, "%s_%s_%s" % (lhs, op, rhs))


def test_ctypes_structs_match_header_layout(tmp_path):
    """The ctypes mirrors in dgl/_ffi.py have the C layout of include/dglmi.h
    (sizes and field offsets, compiled with gcc here)."""
    import ctypes
    import os
    import subprocess
    from dgl import _ffi
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fields = {"DGLMICsr": (_ffi.CSR, [f[0] for f in _ffi.CSR._fields_]),
              "DGLMIGraph": (_ffi.Graph, [f[0] for f in _ffi.Graph._fields_]),
              "DGLMIArray": (_ffi.Array, [f[0] for f in _ffi.Array._fields_]),
              "DGLMIEpilogue": (_ffi.Epilogue, [f[0] for f in _ffi.Epilogue._fields_]),
              "DGLMIRgcnState": (_ffi.RgcnState, [f[0] for f in _ffi.RgcnState._fields_])}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "dglmi.h"', "int main(void) {"]
    for cname, (_, names) in fields.items():
        lines.append('printf("%%s %%zu\\n", "%s", sizeof(%s));' % (cname, cname))
        for f in names:
            lines.append('printf("%%s.%%s %%zu\\n", "%s", "%s", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().split("\n") if l)
    for cname, (cls, names) in fields.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f in names:
            assert int(got["%s.%s" % (cname, f)]) == getattr(cls, f).offset, (cname, f)


def test_64bit_graph_selection():
    """graph_index.py:941-952 switches to int64 ids at 2^31 nodes or edges.  Device
    node ids stay int32, so 2^31 nodes raise DGLError; 2^31 edges (or asbits(64))
    select the 64-bit layout: int64 offsets and edge ids (checked on the GPU in
    tests/test_int64_gpu.py)."""
    from dgl.graph_index import device_block_gidx
    g = GraphIndex(2 ** 31)
    assert g.bits_needed() == 64
    with pytest.raises(dgl.DGLError, match="2\\^31 or more nodes"):
        g.get_immutable_gidx("cuda:0")
    tiny = th.zeros(1, dtype=th.int32)
    with pytest.raises(dgl.DGLError, match="2\\^31 or more nodes"):
        device_block_gidx(2 ** 31, 4, tiny, tiny)
    assert GraphIndex(2 ** 31 - 2).bits_needed() == 32
    small = GraphIndex(3)
    small.add_edges([0, 1], [1, 2])
    assert small.device_bits() == 32
    wide = small.asbits(64)
    assert wide.device_bits() == 64 and small.device_bits() == 32
    assert wide.number_of_edges() == 2 and wide.asbits(32).device_bits() == 32
    with pytest.raises(dgl.DGLError, match="Invalid bit width"):
        small.asbits(16)
    from dgl.graph import _PartialIndex
    assert _PartialIndex(4, [0], [1], [2 ** 31]).bits_needed() == 64
    assert _PartialIndex(4, [0], [1], [5]).bits_needed() == 32


def test_rgcn_fused_ok_matches_the_kernel_rule():
    """dgl.kernel.rgcn_fused_ok restates hack_kernels.hip rgcn_fused_ok (20480 LDS floats
    of weights): C5's 4 relations + self-loop at 64 -> 64 fit, a sixth matrix does not."""
    from dgl import kernel as K
    assert K.rgcn_fused_ok(64, 64, 5) and not K.rgcn_fused_ok(64, 64, 6)
    assert K.rgcn_fused_ok(64, 128, 2) and not K.rgcn_fused_ok(64, 128, 3)
    assert K.rgcn_fused_ok(64, 32, 10) and not K.rgcn_fused_ok(64, 32, 11)
    assert not K.rgcn_fused_ok(32, 64, 1) and not K.rgcn_fused_ok(64, 129, 1)


def test_gatconv_fused_route_limits():
    """GATConv takes the fused kernels only where they apply: 32-bit device CSRs, and
    with attention dropout in training gathered tables below 2^31 elements (the
    dropout walks have 32-bit offsets only, capi.cpp gat_set_dropout), a plain
    nn.Dropout below p = 1 and, for the module's own mask, edge ids that index it."""
    from types import SimpleNamespace
    import torch
    from dgl.nn.pytorch import GATConv, FusedGATConv
    g32 = SimpleNamespace(in_csr=SimpleNamespace(bits=32), eid_perm=True)
    g64 = SimpleNamespace(in_csr=SimpleNamespace(bits=64), eid_perm=True)
    gview = SimpleNamespace(in_csr=SimpleNamespace(bits=32), eid_perm=False)
    big = (1 << 31) // 64
    for mask in ("module", "hashed"):
        conv = GATConv(16, 8, 8, attn_drop=0.5)
        conv.attn_drop_mask = mask
        conv.train()
        assert conv._fused_route(g32, big - 1) and not conv._fused_route(g32, big)
        assert not conv._fused_route(g64, 10)
        # the module's keep words are indexed by edge id: a view whose CSR data are not
        # its own edge ids takes the composition; the hashed mask does not care
        assert conv._fused_route(gview, 10) == (mask == "hashed")
        conv.eval()
        assert conv._fused_route(g32, big)
        conv.use_fused = False
        assert not conv._fused_route(g32, 10)
    # p = 1 (every weight dropped) and a dropout module of another type: the composition
    conv = GATConv(16, 8, 8, attn_drop=1.0).train()
    assert not conv._fused_route(g32, 10)
    conv = GATConv(16, 8, 8, attn_drop=0.5).train()
    conv.attn_drop = torch.nn.AlphaDropout(0.5)
    assert not conv._fused_route(g32, 10)
    # FusedGATConv never applies attn_drop (fusedGatConv.py:80,152): no dropout limits
    conv = FusedGATConv(16, 8, 8, attn_drop=0.5).train()
    assert conv._fused_route(g32, big) and conv._fused_route(gview, 10)
    assert not conv._fused_route(g64, 10)
