"""The five BASELINE.json configs at their FULL sizes on one MI355X (synthetic
graphs with the configs' node and edge counts -- the datasets need downloads).

Small configs are checked exactly against fp64 restatements; at the large ones
the checks are the size-independent kind SURVEY §8(c) asks for: two independent
code paths of the engine against each other (fused vs unfused GAT, the Python
R-GCN path vs the C entry with its own GEMM), a checksum of checksums, and
fp64 recomputation of sampled destination rows with a bound scaled by the row's
absolute mass (fp32 summation order differs from any reference order)."""
import pytest
import torch as th

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _chung_lu(n, m, alpha, seed, self_loops=False):
    g = th.Generator(device=DEV)
    g.manual_seed(seed)
    w = th.arange(1, n + 1, device=DEV, dtype=th.float64).pow(-alpha)
    w = w[th.randperm(n, generator=g, device=DEV)].float()
    src = th.multinomial(w, m, replacement=True, generator=g).to(th.int32)
    dst = th.multinomial(w, m, replacement=True, generator=g).to(th.int32)
    if self_loops:
        ar = th.arange(n, device=DEV, dtype=th.int32)
        src, dst = th.cat([src, ar]), th.cat([dst, ar])
    return src, dst


def _sample_rows(gidx, rows):
    """(segment id, source id, edge id) of the in-edges of `rows`, in-CSR order."""
    ip = gidx.in_csr.indptr.long()
    beg, end = ip[rows], ip[rows + 1]
    lens = end - beg
    seg = th.repeat_interleave(th.arange(rows.numel(), device=DEV), lens)
    pos = th.repeat_interleave(beg - th.cumsum(lens, 0) + lens, lens) + \
        th.arange(int(lens.sum()), device=DEV)
    return seg, gidx.in_csr.indices.long()[pos], gidx.in_csr.data.long()[pos]


def test_c1_cora_gcn_two_layers_exact():
    """C1: 2-layer GraphConv 1433 -> 16 -> 7 on a Cora-size graph (2,708 nodes,
    10,556 edges + self-loops), forward and every gradient vs dense fp64."""
    import dgl
    from dgl.nn.pytorch import GraphConv
    n = 2708
    src, dst = _chung_lu(n, 10556, 0.5, 1, self_loops=True)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    x = (th.rand(n, 1433, device=DEV) < 0.01).float()
    l1, l2 = GraphConv(1433, 16, activation=th.relu).to(DEV), GraphConv(16, 7).to(DEV)
    out = l2(g, l1(g, x))
    out.pow(2).sum().backward()
    A = th.zeros(n, n, dtype=th.float64, device=DEV)
    A.index_put_((dst.long(), src.long()), th.ones(src.numel(), dtype=th.float64, device=DEV),
                 accumulate=True)
    dout = A.sum(0).clamp(min=1).pow(-0.5)
    din = A.sum(1).clamp(min=1).pow(-0.5)
    An = din[:, None] * A * dout[None, :]
    p = [q.detach().double().requires_grad_() for q in (l1.weight, l1.bias, l2.weight, l2.bias)]
    ref = An @ (th.relu(An @ (x.double() @ p[0]) + p[1]) @ p[2]) + p[3]
    ref.pow(2).sum().backward()
    th.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4)
    for a, b in zip((l1.weight, l1.bias, l2.weight, l2.bias), p):
        th.testing.assert_close(a.grad.double(), b.grad, rtol=1e-3, atol=1e-3)


def test_c2_arxiv_graphconv_fwd_bwd():
    """C2: GraphConv 128 -> 128 on an ogbn-arxiv-size graph (169,343 / 1,166,243),
    forward, grad X and grad W vs fp64 torch.sparse."""
    import dgl
    from dgl.nn.pytorch import GraphConv
    n, m = 169_343, 1_166_243
    src, dst = _chung_lu(n, m, 0.8, 2)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    x = th.randn(n, 128, device=DEV, requires_grad=True)
    conv = GraphConv(128, 128).to(DEV)
    out = conv(g, x)
    go = th.randn_like(out)
    out.backward(go)
    s, d = src.long(), dst.long()
    ones = th.ones(m, dtype=th.float64, device=DEV)
    dout = th.zeros(n, dtype=th.float64, device=DEV).index_add_(0, s, ones).clamp(min=1).pow(-0.5)
    din = th.zeros(n, dtype=th.float64, device=DEV).index_add_(0, d, ones).clamp(min=1).pow(-0.5)
    A = th.sparse_coo_tensor(th.stack([d, s]), din[d] * dout[s], (n, n)).coalesce()
    x64 = x.detach().double().requires_grad_()
    w64 = conv.weight.detach().double().requires_grad_()
    ref = th.sparse.mm(A, x64) @ w64 + conv.bias.detach().double()
    ref.backward(go.double())
    mass = th.sparse.mm(A, x64.detach().abs()) @ w64.detach().abs()
    assert ((out.double() - ref).abs() <= 1e-4 + 1e-5 * mass).all()
    th.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=1e-4)
    th.testing.assert_close(conv.weight.grad.double(), w64.grad, rtol=1e-4, atol=1e-2)


def test_c3_reddit_gat_fused_vs_unfused_and_sampled_fp64():
    """C3: GATConv(602, 8, 8 heads) on a Reddit-size graph (232,965 / 114,615,892):
    the fused kernels vs the unfused composition (u_add_v -> edge_softmax ->
    u_mul_e_sum) in outputs and parameter gradients, and 128 sampled destination
    rows recomputed in fp64."""
    import dgl
    from dgl.nn.pytorch import GATConv
    n, m = 232_965, 114_615_892
    src, dst = _chung_lu(n, m, 0.6, 3)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    del src, dst
    x = th.randn(n, 602, device=DEV) / 8
    th.manual_seed(0)
    conv = GATConv(602, 8, 8).to(DEV)
    res = {}
    for fused in (True, False):
        conv.use_fused = fused
        conv.zero_grad()
        out = conv(g, x)
        out.pow(2).sum().backward()
        res[fused] = (out.detach(), [p.grad.clone() for p in conv.parameters()])
    th.testing.assert_close(res[True][0], res[False][0], rtol=1e-4, atol=1e-5)
    for a, b in zip(res[True][1], res[False][1]):
        th.testing.assert_close(a, b, rtol=2e-3, atol=1e-3)
    # fp64 restatement of gatconv.py:143-157 on sampled destination rows
    gidx = g._graph.get_immutable_gidx(DEV)
    rows = th.randint(0, n, (128,), device=DEV)
    seg, us, _ = _sample_rows(gidx, rows)
    W = conv.fc.weight.detach().double()
    ft_u = (x[us].double() @ W.t()).view(-1, 8, 8)
    ft_v = (x[rows].double() @ W.t()).view(-1, 8, 8)
    el = (ft_u * conv.attn_l.detach().double()).sum(-1)
    er = (ft_v * conv.attn_r.detach().double()).sum(-1)[seg]
    e = th.nn.functional.leaky_relu(el + er, 0.2)
    emax = th.full((128, 8), -1e300, dtype=th.float64, device=DEV).index_reduce(0, seg, e, "amax")
    a = (e - emax[seg]).exp()
    a = a / th.zeros(128, 8, dtype=th.float64, device=DEV).index_add_(0, seg, a)[seg]
    ref = th.zeros(128, 8, 8, dtype=th.float64, device=DEV).index_add_(0, seg, a[..., None] * ft_u)
    th.testing.assert_close(res[True][0][rows].double(), ref, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("H", [1, 2, 4, 8])
def test_c3_edge_softmax_full_size(H, monkeypatch):
    """Edge softmax on the C3 graph at full size, forward and backward: on the in-CSR
    position view the H <= 4 four-values-per-lane walk against the one-position walk
    (DGLMI_SOFTMAX_QUAD=0); on the graph itself (edge-id order) the packed row
    statistics against the two arrays (DGLMI_SOFTMAX_PACK=0, the same bits); and 128
    sampled destination rows of both recomputed in fp64."""
    import dgl
    from dgl import kernel as K
    n, m = 232_965, 114_615_892
    src, dst = _chung_lu(n, m, 0.6, 3)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    del src, dst
    gidx = g._graph.get_immutable_gidx(DEV)
    view = gidx.position_view("in")
    gen = th.Generator(device=DEV).manual_seed(H)
    s = th.randn(m, H, device=DEV, generator=gen) * 3
    ga = th.randn(m, H, device=DEV, generator=gen)

    def run(gi, env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        a, gs = th.empty_like(s), th.empty_like(s)
        K.edge_softmax_forward(gi, s, a)
        K.edge_softmax_backward(gi, a, ga, gs)
        return a, gs
    rows = th.randint(0, n, (128,), device=DEV)
    seg, _, eids = _sample_rows(gidx, rows)
    ip = gidx.in_csr.indptr.long()
    pos = th.cat([th.arange(int(ip[r]), int(ip[r + 1]), device=DEV) for r in rows.tolist()])

    def check(a, gs, idx, x):
        # fp64 softmax and its backward over the sampled rows' edges (idx: where they sit)
        e = x[idx].double()
        emax = th.full((128, H), -1e300, dtype=th.float64, device=DEV).index_reduce(0, seg, e, "amax")
        w = (e - emax[seg]).exp()
        w = w / th.zeros(128, H, dtype=th.float64, device=DEV).index_add_(0, seg, w)[seg]
        th.testing.assert_close(a[idx].double(), w, rtol=1e-5, atol=1e-7)
        g64 = ga[idx].double()
        S = th.zeros(128, H, dtype=th.float64, device=DEV).index_add_(0, seg, w * g64)
        th.testing.assert_close(gs[idx].double(), w * g64 - w * S[seg], rtol=1e-4, atol=1e-6)

    # position view: the logits in walk order (s is read as position-ordered there)
    monkeypatch.setenv("DGLMI_SOFTMAX_OWNED", "1")
    a1, g1 = run(view, {"DGLMI_SOFTMAX_QUAD": "1"})
    a0, g0 = run(view, {"DGLMI_SOFTMAX_QUAD": "0"})
    th.testing.assert_close(a1, a0, rtol=1e-5, atol=1e-7)
    th.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-6)
    check(a1, g1, pos, s)
    del a0, g0
    # the graph in edge-id order
    b1, h1 = run(gidx, {"DGLMI_SOFTMAX_QUAD": "1", "DGLMI_SOFTMAX_PACK": "1"})
    b0, h0 = run(gidx, {"DGLMI_SOFTMAX_QUAD": "0", "DGLMI_SOFTMAX_PACK": "0"})
    assert th.equal(b1, b0) and th.equal(h1, h0)
    check(b1, h1, eids, s)


def test_c4_rmat_copy_u_sum_and_partition():
    """C4 on one GPU: copy_u_sum over the 10 M / 200 M RMAT graph (checksum of
    checksums + 2,048 sampled rows in fp64), and the 8-way device partition:
    within its edge cap, fewer cut edges and halo rows than the contiguous split."""
    import bench
    from dgl import distributed as D
    from dgl import kernel as K
    from dgl.graph_index import device_block_gidx
    src, dst, x = bench.c4_workload(DEV)
    n = bench.C4_NODES
    gidx = device_block_gidx(n, n, src, dst)
    out = th.empty(n, 64, device=DEV)
    K.copy_reduce("sum", gidx, 0, x, out)
    outdeg = th.bincount(src.long(), minlength=n).double()
    expect = th.zeros(64, dtype=th.float64, device=DEV)
    for lo in range(0, n, 1 << 22):
        expect += (outdeg[lo:lo + (1 << 22), None] * x[lo:lo + (1 << 22)].double()).sum(0)
    got = out.double().sum(0)
    assert float((got - expect).abs().max() / expect.abs().max()) < 1e-6
    rows = th.randint(0, n, (2048,), device=DEV)
    seg, us, _ = _sample_rows(gidx, rows)
    exact = th.zeros(2048, 64, dtype=th.float64, device=DEV).index_add_(0, seg, x[us].double())
    mass = th.zeros(2048, 64, dtype=th.float64, device=DEV).index_add_(0, seg, x[us].double().abs())
    assert ((out[rows].double() - exact).abs() <= 1e-5 + 1e-6 * mass).all()
    assign, info = D.partition_labelprop(gidx, 8, rounds=24)
    w = (gidx.in_csr.degrees() + 1).long()
    assert max(info["loads"]) <= 1.05 * float(w.sum()) / 8 + 1
    st = D.partition_stats(src, dst, assign, 8)
    ct = D.partition_stats(src, dst, D.contiguous_parts_device(w.int(), 8), 8)
    assert st["cut_edges"] < ct["cut_edges"] and sum(st["halo_rows"]) < sum(ct["halo_rows"])


def _sample_out_rows(gidx, rows):
    """(segment id, destination id, edge id) of the out-edges of `rows`, out-CSR order."""
    ip = gidx.out_csr.indptr.long()
    beg, end = ip[rows], ip[rows + 1]
    lens = end - beg
    seg = th.repeat_interleave(th.arange(rows.numel(), device=DEV), lens)
    pos = th.repeat_interleave(beg - th.cumsum(lens, 0) + lens, lens) + \
        th.arange(int(lens.sum()), device=DEV)
    return seg, gidx.out_csr.indices.long()[pos], gidx.out_csr.data.long()[pos]


def _typed_rows(a, t, W, transpose=False):
    """Row i of the result is a[i] @ W[t[i]] (or @ W[t[i]]^T): one GEMM per relation,
    never an (E, F, F) tensor of per-edge weights."""
    out = th.zeros(a.shape[0], W.shape[1] if transpose else W.shape[2], dtype=a.dtype,
                   device=a.device)
    for r in range(W.shape[0]):
        sel = t == r
        out[sel] = a[sel] @ (W[r].t() if transpose else W[r])
    return out


def _rows_with_hubs(deg, k_hub, k_rand, n):
    """The k_hub highest-degree rows (hub rows span many work shares) + random rows."""
    return th.cat([th.topk(deg, k_hub).indices, th.randint(0, n, (k_rand,), device=DEV)])


def test_c5_rgcn_fused_route_full_size():
    """C5 at full size (5 M nodes / 80 M typed edges, 4 relations, 64 -> 64, self-loop
    and bias, norm = 1 / in-degree) -- the configuration the bench's C5 line times.

    (1) RelGraphConv on the fused route (DGLMIRgcnLayer1Ex / BackwardEx with the prepared
    state: tile queues over ~156 K row tiles, ordered per-group carries, hub rows spanning
    many shares) vs the GEMM + typed-gather route: output, input gradient and every
    parameter gradient.
    (2) The C entries on a prepared state (layers 4 and 6) vs the restatement of the
    hack's layer-1 formula (oracle/hack_ref.c: ret[v] = sum_e norm_e h[u] W[t_e], plus
    RelGraphConv's bias and self-loop; binary_reduce_impl.cu:1082-1194) in fp64: 256
    destination rows (the 32 largest in-degrees among them) for the output, 256 source
    rows (the 32 largest out-degrees) for the input gradient, and the whole relation and
    self-loop weight gradients.  Bounds scale with the absolute mass of each sum."""
    import dgl
    from dgl import kernel as K
    from dgl.nn.pytorch import RelGraphConv
    n, m, R = 5_000_000, 80_000_000, 4
    src, dst = _chung_lu(n, m, 0.5, 5)
    gen = th.Generator(device=DEV)
    gen.manual_seed(8)
    et = th.randint(0, R, (m,), device=DEV, generator=gen)
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    indeg = th.bincount(dst.long(), minlength=n)
    outdeg = th.bincount(src.long(), minlength=n)
    norm = (1.0 / indeg.clamp(min=1).float())[dst.long()].view(-1, 1)
    del src, dst
    th.manual_seed(0)
    conv = RelGraphConv(64, 64, R, "basis", num_bases=R, self_loop=True).to(DEV)
    with th.no_grad():
        conv.h_bias.uniform_(-1, 1)
    h = th.randn(n, 64, device=DEV, requires_grad=True)
    go = th.randn(n, 64, device=DEV)
    params = [h] + list(conv.parameters())
    res = {}
    for fused in (True, False):
        conv.use_fused = fused
        out = conv(g, h, et, norm)
        if fused:
            assert g._graph.__dict__.get("_rgcn_fused") is not None  # the fused route ran
        res[fused] = (out.detach(), th.autograd.grad(out, params, go))
        del out
    th.testing.assert_close(res[True][0], res[False][0], rtol=1e-4, atol=1e-4)
    for a, b in zip(res[True][1], res[False][1]):  # long fp32 sums in two orders
        assert (a - b).abs().max().item() <= 1e-3 + 1e-4 * b.abs().max().item()
    del res
    g._graph.__dict__.pop("_rgcn_fused", None)
    # (2) the C entries on prepared state vs the fp64 formula
    gidx = g._graph.get_immutable_gidx(DEV)
    gidx.__dict__.pop("_rgcn_state", None)
    et32 = et.int()
    hd = h.detach()
    Wr = conv._relation_weights().detach().contiguous()
    lw = conv.loop_weight.detach().contiguous()
    bias = conv.h_bias.detach().contiguous()
    nf = norm.reshape(-1).contiguous()
    rows = _rows_with_hubs(indeg, 32, 224, n)
    seg, us, es = _sample_rows(gidx, rows)
    W64 = Wr.double()
    nu = nf[es, None].double()
    msg = _typed_rows(hd[us].double(), et[es], W64) * nu
    amsg = _typed_rows(hd[us].double().abs(), et[es], W64.abs()) * nu
    ref = th.zeros(256, 64, dtype=th.float64, device=DEV).index_add_(0, seg, msg) + \
        hd[rows].double() @ lw.double() + bias.double()
    mass = th.zeros(256, 64, dtype=th.float64, device=DEV).index_add_(0, seg, amsg) + \
        hd[rows].double().abs() @ lw.double().abs() + bias.double().abs()
    srows = _rows_with_hubs(outdeg, 32, 224, n)
    sseg, vs, ses = _sample_out_rows(gidx, srows)
    gmsg = go[vs].double() * nf[ses, None].double()
    gh_ref = th.zeros(256, 64, dtype=th.float64, device=DEV).index_add_(
        0, sseg, _typed_rows(gmsg, et[ses], W64, True)) + go[srows].double() @ lw.double().t()
    gh_mass = th.zeros(256, 64, dtype=th.float64, device=DEV).index_add_(
        0, sseg, _typed_rows(gmsg.abs(), et[ses], W64.abs(), True)) + \
        go[srows].double().abs() @ lw.double().abs().t()
    # the whole weight gradients in fp64: gW[t] = sum_{e of t} norm_e h[u]^T go[v], chunked
    ic = gidx.in_csr
    gw_ref = th.zeros(R, 64, 64, dtype=th.float64, device=DEV)
    gw_mass = th.zeros_like(gw_ref)
    for lo in range(0, m, 1 << 22):
        u = ic.indices[lo:lo + (1 << 22)].long()
        v = ic.rows[lo:lo + (1 << 22)].long()
        e = ic.data[lo:lo + (1 << 22)].long()
        t = et[e]
        a, b = hd[u].double(), go[v].double() * nf[e, None].double()
        for r in range(R):
            sel = t == r
            gw_ref[r] += a[sel].t() @ b[sel]
            gw_mass[r] += a[sel].abs().t() @ b[sel].abs()
        del u, v, e, t, a, b
    gl_ref = hd.double().t() @ go.double()
    gl_mass = hd.double().abs().t() @ go.double().abs()
    for layers in (4, 6):
        K.rgcn_prepare(gidx, nf, R, layers=layers, etypes=et32)
        ret = th.full((n, 64), float("nan"), device=DEV)
        K.rgcn_layer1_ex(gidx, hd, Wr, nf, ret, loop_weight=lw, bias=bias, etypes=et32)
        assert ((ret[rows].double() - ref).abs() <= 1e-5 + 1e-5 * mass).all(), layers
        assert not th.isnan(ret).any()
        del ret
        gh = th.full((n, 64), float("nan"), device=DEV)
        gw, gl = th.full_like(Wr, float("nan")), th.full_like(lw, float("nan"))
        K.rgcn_layer1_backward_ex(gidx, hd, Wr, nf, lw, go, gh, gw, gl, etypes=et32)
        assert ((gh[srows].double() - gh_ref).abs() <= 1e-5 + 1e-5 * gh_mass).all(), layers
        assert not th.isnan(gh).any()
        del gh
        assert ((gw.double() - gw_ref).abs() <= 2e-4 + 1e-6 * gw_mass).all(), layers
        assert ((gl.double() - gl_ref).abs() <= 2e-4 + 1e-6 * gl_mass).all(), layers
    gidx.__dict__.pop("_rgcn_state").release()
