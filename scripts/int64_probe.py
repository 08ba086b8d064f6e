"""64-bit graph probe: what the int64 offsets / edge ids cost, and a
graph past 2^31 edges on one MI355X.

A. M1 (RMAT scale 23, 100 M edges, F = 64) in the int32 layout and forced to the
   64-bit layout (GraphIndex.asbits(64)): update_all(copy_u, sum) forward and the
   source gradient, HIP events on the current stream, median of 20; outputs
   compared bit for bit.
B. RMAT scale 26 (67 M nodes), 2^31 + 2^28 edges (ids permuted), F = 64: device
   ingestion time (two batched stable COO -> CSR passes + row expansion), then the
   same forward / backward timings.

Prints one JSON object.
"""
import json
import os
import sys
import time

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, ROOT)

import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from bench import rmat_edges  # noqa: E402

DEV = th.device("cuda:0")


def timed(fn_, reps=20, warm=3):
    for _ in range(warm):
        fn_()
    ts = []
    for _ in range(reps):
        a, b = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
        a.record()
        fn_()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def fwd_bwd(g, x, reps=20):
    g.ndata["x"] = x
    fwd = timed(lambda: g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o")), reps)
    out = g.ndata["o"]
    xr = x.clone().requires_grad_()
    g.ndata["x"] = xr
    g.update_all(fn.copy_u("x", "m"), fn.sum("m", "o"))
    y = g.ndata["o"]
    go = th.ones_like(y)
    bwd = timed(lambda: th.autograd.grad(y, xr, go, retain_graph=True), reps)
    (gx,) = th.autograd.grad(y, xr, go, retain_graph=True)
    return fwd, bwd, out, gx


def permuted_rmat(scale, m, seed):
    n = 1 << scale
    src, dst = rmat_edges(scale, m, seed=seed, device=DEV)
    gp = th.Generator(device=DEV)
    gp.manual_seed(1)
    perm = th.randperm(n, generator=gp, device=DEV).to(th.int32)
    step = 1 << 28
    for b in range(0, m, step):  # in place, chunked (no 8-byte copy of the whole list)
        src[b:b + step] = perm[src[b:b + step].long()]
        dst[b:b + step] = perm[dst[b:b + step].long()]
    del perm
    return n, src, dst


def main():
    res = {}
    # A. M1, both layouts
    n, src, dst = permuted_rmat(23, 100_000_000, seed=1234)
    g32 = dgl.DGLGraph.from_device_coo(src, dst, n)
    g64 = dgl.DGLGraph(g32._graph.asbits(64))
    x = th.rand(n, 64, device=DEV) * 2 - 1
    th.cuda.synchronize()
    t0 = time.time()
    g64._graph.get_immutable_gidx(DEV)
    th.cuda.synchronize()
    build64 = time.time() - t0
    t0 = time.time()
    g32._graph.get_immutable_gidx(DEV)
    th.cuda.synchronize()
    build32 = time.time() - t0
    f32, b32, o32, gx32 = fwd_bwd(g32, x)
    f64, b64, o64, gx64 = fwd_bwd(g64, x)
    res["M1"] = {"edges": 100_000_000, "feat": 64,
                 "int32": {"build_s": build32, "fwd_ms": f32, "bwd_ms": b32},
                 "int64": {"build_s": build64, "fwd_ms": f64, "bwd_ms": b64},
                 "bit_identical": bool(th.equal(o32, o64) and th.equal(gx32, gx64))}
    print(json.dumps(res), flush=True)
    del g32, g64, o32, o64, gx32, gx64, src, dst, x
    th.cuda.empty_cache()

    # B. past 2^31 edges
    m = (1 << 31) + (1 << 28)
    t0 = time.time()
    n, src, dst = permuted_rmat(26, m, seed=99)
    th.cuda.synchronize()
    gen_s = time.time() - t0
    g = dgl.DGLGraph.from_device_coo(src, dst, n)
    t0 = time.time()
    gidx = g._graph.get_immutable_gidx(DEV)
    th.cuda.synchronize()
    build = time.time() - t0
    del src, dst  # (the graph keeps its COO: 19 GB)
    x = th.rand(n, 64, device=DEV) * 2 - 1
    f, b, out, gx = fwd_bwd(g, x, reps=5)
    # checksums of checksums (fp64): sum_v out[v] = sum_u outdeg(u) x[u], and the gradient
    outdeg = gidx.out_csr.degrees().double()
    indeg = gidx.in_csr.degrees().double()
    c1 = float(((out.double().sum(0) - (outdeg[:, None] * x.double()).sum(0)).abs().max()
                / (outdeg[:, None] * x.double().abs()).sum(0).max()))
    c2 = float(((gx.double().sum(0) - indeg.sum()).abs() / indeg.sum()).max())
    res["big"] = {"nodes": n, "edges": m, "feat": 64, "num_bits": gidx.num_bits,
                  "generate_s": gen_s, "build_s": build,
                  "fwd_ms": f, "bwd_ms": b, "fwd_edges_per_s": m / (f * 1e-3),
                  "bwd_edges_per_s": m / (b * 1e-3),
                  "checksum_rel_err": c1, "grad_checksum_rel_err": c2,
                  "hbm_allocated_GB": th.cuda.max_memory_allocated() / 1e9}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
