#!/usr/bin/env python3
"""Headline benchmark: GCN copy_u_sum (g-SpMM) on a 100M-edge RMAT graph.

Metric (BASELINE.json): edges/sec + achieved HBM GB/s, GCN copy_u_sum on a
100M-edge graph, 1/2/4/8 MI355X.

Workload M1: RMAT (a,b,c,d) = (0.57, 0.19, 0.19, 0.05),
scale 23 (N = 8,388,608), E = 100,000,000, vertex ids randomly permuted,
duplicates and self-loops kept, X ~ U(-1, 1) of shape (N, 64) fp32, int32
dst-major CSR.  Generated on the GPU (seeded), CSRs built on the GPU.

A step = one copy_u_sum pass (DGLGraph.update_all(copy_u, sum) lowers to
exactly this call) over the resident graph: out[v] = sum_{u->v} X[u].

Multi-GPU (torchrun, one process per GPU): weak scaling.  The global graph
has N x 100M edges (RMAT scale 23 + log2 N); every rank owns a contiguous
block of destination rows with all their in-edges (1-D row partition, the
halo-subgraph semantics of graph_op.cc:403-509 with num_hops = 1) and holds
the source features replicated (DESIGN.md "Multi-GPU"), so the timed SpMM
has no data-path collective.  `value` = all ranks' edges / max-over-ranks time.

cpu_baseline: the reference's CPU algorithm (out-CSR traversal, OpenMP over
source rows, `omp atomic` scatter; oracle/dgl_ref.c) on a bounded sample of
the same graph, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "dgl-hack_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch as th  # noqa: E402

RMAT = (0.57, 0.19, 0.19, 0.05)
SCALE = 23
EDGES_PER_GPU = 100_000_000
FEAT = 64
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def rmat_edges(scale, num_edges, seed, device, chunk=25_000_000):
    """RMAT edge list on the GPU (int32 src, dst), unpermuted ids."""
    a, b, c, _ = RMAT
    gen = th.Generator(device=device)
    gen.manual_seed(seed)
    srcs, dsts = [], []
    done = 0
    while done < num_edges:
        cnt = min(chunk, num_edges - done)
        s = th.zeros(cnt, dtype=th.int32, device=device)
        d = th.zeros(cnt, dtype=th.int32, device=device)
        for lvl in range(scale):
            r = th.rand(cnt, generator=gen, device=device)
            sb = r > (a + b)
            db = ((r > a) & (r <= a + b)) | (r > a + b + c)
            s |= sb.to(th.int32) << lvl
            d |= db.to(th.int32) << lvl
        srcs.append(s)
        dsts.append(d)
        done += cnt
    return th.cat(srcs), th.cat(dsts)


def build_workload(world, rank, device, edges_per_gpu=EDGES_PER_GPU, scale0=SCALE):
    scale = scale0 + int(round(math.log2(world)))
    n = 1 << scale
    m = edges_per_gpu * world
    t0 = time.time()
    src, dst = rmat_edges(scale, m, seed=1234, device=device)
    gp = th.Generator(device=device)
    gp.manual_seed(1)
    perm = th.randperm(n, generator=gp, device=device).to(th.int32)
    src = perm[src.long()]
    dst = perm[dst.long()]
    del perm
    lo = n * rank // world
    hi = n * (rank + 1) // world
    if world > 1:
        keep = (dst >= lo) & (dst < hi)
        src, dst = src[keep], dst[keep] - lo
    gx = th.Generator(device=device)
    gx.manual_seed(2)
    x = th.rand(n, FEAT, generator=gx, device=device) * 2 - 1
    th.cuda.synchronize()
    log("graph generated: scale %d, %d edges total, rank rows [%d, %d), %d local edges (%.1fs)"
        % (scale, m, lo, hi, src.shape[0], time.time() - t0))
    return n, hi - lo, src.contiguous(), dst.contiguous(), x


def make_local_graph(n_src, n_dst, src, dst, device):
    """Local in-CSR (rows = owned dst, cols = global src) built on the GPU."""
    from dgl.graph_index import device_block_gidx
    g = device_block_gidx(n_src, n_dst, src, dst)
    return g, (g.out_csr.indptr, g.out_csr.indices)


def cpu_baseline(o_ptr, o_idx, x, n_dst, budget_s=20.0, sample_edges=None):
    """Reference CPU algorithm on the M1 graph (or its leading source rows when
    `sample_edges` is given), passes repeated until `budget_s` is spent (>= 1 pass)."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or O.max_threads()
    ptr = o_ptr.cpu().numpy()
    rows = ptr.shape[0] - 1
    if sample_edges is not None:
        rows = max(1, min(rows, int(np.searchsorted(ptr, sample_edges, side="right")) - 1))
    e = int(ptr[rows])
    idx = o_idx[:e].cpu().numpy().astype(np.int32)
    xs = np.ascontiguousarray(x[:rows].cpu().numpy())  # features of the sampled source rows
    ptr_s = ptr[:rows + 1].astype(np.int32)
    times = []
    t_start = time.time()
    for it in range(5):
        t0 = time.time()
        O.copy_src_sum_i32(rows, ptr_s, idx, xs, n_dst, threads)
        times.append(time.time() - t0)
        if time.time() - t_start > budget_s:
            break
    t = float(np.median(times))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": e / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpus": os.cpu_count(),
            "sample": "reference CPU algorithm (oracle/dgl_ref.c ref_copy_src_sum_i32: out-CSR, "
                      "OpenMP over src rows, omp-atomic scatter, zero fill of all %d dst rows) on "
                      "%d source rows (%d edges) of the M1 graph, F=%d, median of %d pass(es), "
                      "%d OpenMP threads" % (n_dst, rows, e, FEAT, len(times), threads),
            "seconds_per_pass": t}


def load_pmc_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get("bytes_per_launch")
    except Exception:
        return None


def _max_over_ranks(v, dist, cdev):
    """max of a float over all ranks (so every rank takes the same exit path)."""
    if dist is None:
        return float(v)
    t = th.tensor([float(v)], device=cdev, dtype=th.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed(fn, steps, dist, cdev):
    """barrier + sync bracketed wall time of `steps` calls, max over ranks (s)."""
    if dist is not None:
        dist.barrier()
    th.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    th.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t
    if dist is not None:
        v = th.tensor([el], device=cdev, dtype=th.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        el = float(v.item())
    return el


def measure_exchange(part, x, out_ref, args, dist, cdev, device, edges_total):
    """copy_u_sum with the source rows NOT replicated: each step first fetches
    the halo rows with one all-to-all-v (RCCL over xGMI), then aggregates over
    the local [owned | halo] block.  SURVEY §8(e): the with-exchange line."""
    from dgl import distributed as D
    from dgl import kernel as K
    x_full = th.empty(part.n_inner + part.n_halo, FEAT, device=device)
    x_full[:part.n_inner] = x[part.lo:part.hi]
    send_buf = th.empty(int(part.send_counts.sum()), FEAT, device=device)
    out = th.empty_like(out_ref)
    g = part.gidx()

    def xstep():
        D.halo_exchange_into(x_full, part, None, send_buf)
        K.copy_reduce("sum", g, 0, x_full, out)
    xstep()
    th.cuda.synchronize()
    err = float((out - out_ref).abs().max() / out_ref.abs().max().clamp(min=1e-30))
    err = _max_over_ranks(err, dist, cdev)
    if err > 1e-4:
        raise SystemExit("with-exchange copy_u_sum differs from the replicated one: %g" % err)
    steps = max(1, min(args.steps, 5))
    for _ in range(2):
        xstep()
    el = _timed(xstep, steps, dist, cdev)
    moved = th.tensor([float(part.n_halo) * FEAT * 4], device=cdev, dtype=th.float64)
    halo_max = th.tensor([float(part.n_halo)], device=cdev, dtype=th.float64)
    dist.all_reduce(moved)
    dist.all_reduce(halo_max, op=dist.ReduceOp.MAX)
    ex_el = _timed(lambda: D.halo_exchange_into(x_full, part, None, send_buf), steps, dist, cdev)
    # overlapped: owned-source half of the SpMM while the all-to-all-v is in flight,
    # halo half accumulated in the kernel epilogue (dgl.distributed.aggregate_with_halo)
    x_inner = x[part.lo:part.hi]
    recv = th.empty(part.n_halo, FEAT, device=device)
    tmp = th.empty_like(out)
    out2 = th.empty_like(out)

    def ostep():
        D.aggregate_with_halo(x_inner, part, out2, None, recv, send_buf, tmp)
    ostep()
    th.cuda.synchronize()
    oerr = _max_over_ranks(float((out2 - out_ref).abs().max() / out_ref.abs().max().clamp(min=1e-30)),
                           dist, cdev)
    if oerr > 1e-4:
        raise SystemExit("overlapped with-exchange copy_u_sum differs: %g" % oerr)
    for _ in range(2):
        ostep()
    ov_el = _timed(ostep, steps, dist, cdev)
    return {"value": edges_total * steps / ov_el, "unit": "edges/s",
            "ms_per_step": ov_el * 1e3 / steps,
            "schedule": "halo all-to-all-v overlapped with the owned-source half of the SpMM",
            "sequential_ms_per_step": el * 1e3 / steps,
            "sequential_edges_per_s": edges_total * steps / el,
            "exchange_only_ms": ex_el * 1e3 / steps, "steps": steps,
            "halo_bytes_per_step_all_ranks": float(moved.item()),
            "max_halo_rows_per_rank": int(halo_max.item()),
            "exchange": "all_to_all_single (%s) of halo source rows, then local copy_u_sum"
                        % dist.get_backend(),
            "rel_err_vs_replicated": max(err, oerr)}


def stream_copy_peak(device, nbytes=4 << 30, reps=5):
    """Measured HBM stream rate: device-to-device copy of a 4 GiB buffer,
    (read + write bytes) / time -- BASELINE.md §3's measured peak beside the spec."""
    a = th.empty(nbytes // 4, dtype=th.float32, device=device)
    b = th.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    s, e = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        b.copy_(a)
    e.record()
    th.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def measure_update_all(g, x, out_ref, args):
    """End-to-end DGLGraph.update_all(copy_u, sum) through the Python boundary
    (frame lookup, output allocation, autograd Function, ctypes call)."""
    import dgl.function as fn
    g.ndata["h"] = x
    g.update_all(fn.copy_u("h", "m"), fn.sum("m", "h2"))  # builds + caches the device CSRs
    th.cuda.synchronize()
    if not th.equal(g.ndata["h2"], out_ref):
        raise SystemExit("update_all result differs from the direct kernel call")
    steps = max(1, min(args.steps, 10))
    el = _timed(lambda: g.update_all(fn.copy_u("h", "m"), fn.sum("m", "h2")), steps, None, None)
    return {"ms_per_call": el * 1e3 / steps, "edges_per_sec": g.number_of_edges() * steps / el,
            "path": "DGLGraph.update_all(fn.copy_u, fn.sum) incl. output allocation"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # rehearsal knobs (small graphs, gloo collectives with every rank on one GPU);
    # the headline run uses the defaults
    ap.add_argument("--edges-per-gpu", type=int, default=EDGES_PER_GPU)
    ap.add_argument("--scale", type=int, default=SCALE)
    ap.add_argument("--dist-backend", default="nccl")
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--no-exchange", action="store_true",
                    help="N>1: skip the with-halo-exchange measurement")
    ap.add_argument("--no-update-all", action="store_true",
                    help="N=1: skip the end-to-end DGLGraph.update_all measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    th.cuda.set_device(local)
    device = "cuda:%d" % local
    dist = None
    cdev = device
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=th.device(device))
        else:
            dist.init_process_group(args.dist_backend)
            cdev = "cpu"  # gloo collectives on host tensors

    import dgl  # noqa: F401
    from dgl import kernel as K

    n, n_dst, src, dst, x = build_workload(world, rank, device, args.edges_per_gpu, args.scale)
    t0 = time.time()
    gidx, (o_ptr, o_idx) = make_local_graph(n, n_dst, src, dst, device)
    m_local = src.shape[0]
    th.cuda.synchronize()
    log("CSRs built on device in %.2fs" % (time.time() - t0))
    part = None
    if world > 1 and not args.no_exchange:
        # the same rows planned as a halo partition (owned X rows + halo rows
        # fetched by one all-to-all-v per step), for the with-exchange line
        from dgl import distributed as D
        t0 = time.time()
        bounds = [n * p // world for p in range(world + 1)]
        part = D.build_device_partition(src, dst, bounds, rank)
        part.release_edges()
        th.cuda.synchronize()
        log("halo plan built on device in %.2fs: %d halo rows on rank 0"
            % (time.time() - t0, part.n_halo))
    upd = None
    if world == 1 and not args.no_update_all:
        import dgl
        upd = dgl.DGLGraph.from_device_coo(src, dst, n)
    del src, dst

    out = th.empty(n_dst, FEAT, device=device)

    def step():
        K.copy_reduce("sum", gidx, 0, x, out)

    # correctness spot check on the resident workload: a checksum of checksums is
    # order-independent up to fp32 rounding (sum over rows of out == sum_u outdeg(u) * X[u])
    step()
    th.cuda.synchronize()
    outdeg = th.bincount(gidx.in_csr.indices.long(), minlength=n).double()
    expect = th.zeros(FEAT, dtype=th.float64, device=device)
    for lo in range(0, n, 1 << 22):  # chunked: x.double() of a 2^26-row table is 34 GB
        hi = min(n, lo + (1 << 22))
        expect += (outdeg[lo:hi, None] * x[lo:hi].double()).sum(0)
    got = out.double().sum(0)
    rel = float(((got - expect).abs().max() / expect.abs().max().clamp(min=1)).item())
    rel = _max_over_ranks(rel, dist, cdev)
    log("checksum-of-checksums rel err %.2e (max over ranks)" % rel)
    if rel > 1e-3:
        raise SystemExit("copy_u_sum checksum mismatch: %g" % rel)
    del outdeg, expect, got
    # row-exact spot check: 4096 random rows recomputed with torch gathers (fp64)
    gen = th.Generator(device=device)
    gen.manual_seed(7)
    rows = th.randint(0, n_dst, (4096,), generator=gen, device=device)
    ip = gidx.in_csr.indptr.long()
    beg, end = ip[rows], ip[rows + 1]
    lens = end - beg
    seg = th.repeat_interleave(th.arange(4096, device=device), lens)
    pos = th.repeat_interleave(beg - th.cumsum(lens, 0) + lens, lens) + th.arange(int(lens.sum()), device=device)
    cols = gidx.in_csr.indices.long()[pos]
    xr = x.double()[cols]
    exact = th.zeros(4096, FEAT, dtype=th.float64, device=device).index_add_(0, seg, xr)
    mass = th.zeros(4096, FEAT, dtype=th.float64, device=device).index_add_(0, seg, xr.abs())
    err = (out[rows].double() - exact).abs()
    bad = _max_over_ranks(float((err > 1e-4 + 1e-6 * mass).any()), dist, cdev)
    if bad > 0:
        raise SystemExit("copy_u_sum row check failed: max err %g" % float(err.max()))
    log("row spot check (4096 rows, fp64 torch gathers): max abs err %.2e" % float(err.max()))
    del seg, pos, cols, xr, exact, mass, err

    for _ in range(args.warmup):
        step()
    stream = th.cuda.current_stream()
    ev = [(th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    th.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    th.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    th.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    edges_total = m_local
    if dist is not None:
        t = th.tensor([elapsed], device=cdev, dtype=th.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = th.tensor([kernel_ms], device=cdev, dtype=th.float64)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        kernel_ms = float(k.item())
        e = th.tensor([m_local], device=cdev, dtype=th.float64)
        dist.all_reduce(e)
        edges_total = int(e.item())

    ms_per_step = elapsed * 1000.0 / args.steps
    value = edges_total * args.steps / elapsed
    exch = None
    if part is not None:
        try:
            exch = measure_exchange(part, x, out, args, dist, cdev, device, edges_total)
        except SystemExit as exc:
            # its parity checks agree across ranks (max over ranks) before exiting, so
            # every rank lands here together; the replicated headline still reports
            exch = {"error": str(exc)}
    upd_res = None
    if upd is not None:
        upd_res = measure_update_all(upd, x, out, args)
        del upd
    # algorithmic bytes per launch (per rank): indptr + indices + one
    # gathered 4F-byte source row per edge + one 4F-byte output row per destination
    alg_bytes = 4 * (n_dst + 1) + 4 * m_local + 4 * FEAT * m_local + 4 * FEAT * n_dst
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    compulsory = 4 * (n_dst + 1) + 4 * m_local + 4 * FEAT * n + 4 * FEAT * n_dst
    # the committed PMC summary was measured on the default M1 launch only
    m1 = world == 1 and args.edges_per_gpu == EDGES_PER_GPU and args.scale == SCALE
    pmc = load_pmc_traffic() if m1 else None
    res = {
        "metric": "edges/sec + achieved HBM GB/s, GCN copy_u_sum on 100M-edge graph, 1/2/4/8 MI355X",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic RMAT(0.57,0.19,0.19,0.05) generated on device, ids permuted, "
                "X~U(-1,1) seed 2",
        "config": {"workload": "M1 copy_u_sum: RMAT scale %d, %d edges, feat %d, int32 in-CSR%s"
                               % (args.scale + int(round(math.log2(world))), args.edges_per_gpu * world,
                                  FEAT, "" if world == 1 else
                                  ", %d-way dst-row partition, X replicated" % world),
                   "nodes": n, "edges": args.edges_per_gpu * world, "feat": FEAT,
                   "parallelism": "dst-row partition x%d" % world if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": pmc,
                     "kernel": "k_chunk_reduce + k_chunk_fixup (one copy_u_sum launch pair)",
                     "kernel_ms": kernel_ms, "alg_bytes_per_launch": alg_bytes,
                     "compulsory_bytes_per_launch": compulsory},
        "hbm_gbps_achieved": achieved,
        "edges_per_sec_per_gpu": value / world,
    }
    try:
        peak = stream_copy_peak(device)
        res["roofline"]["measured_stream_copy_GBps"] = peak
        res["roofline"]["stream_copy_method"] = "torch copy_ of a 4 GiB fp32 buffer, (read + write) / time"
    except RuntimeError as exc:  # out of memory on a crowded device: report, don't fail
        res["roofline"]["measured_stream_copy_GBps"] = None
        log("stream copy peak skipped: %r" % exc)
    if pmc:
        # bytes the PMC counters saw leave L2 for the fabric (Infinity Cache + HBM)
        # per launch, moved in the measured kernel time
        fab = pmc / (kernel_ms * 1e-3) / 1e9
        res["roofline"]["traffic_GBps"] = fab
        res["roofline"]["traffic_frac_of_peak"] = fab / HBM_PEAK_GBPS
        res["roofline"]["traffic_note"] = ("2 x FETCH_SIZE + WRITE_SIZE of the M1 launch pair "
                                           "(profiles/pmc_traffic.json, gfx950 wide-read "
                                           "correction); includes Infinity-Cache hits")
    if exch is not None:
        res["with_exchange"] = exch
    if upd_res is not None:
        res["update_all"] = upd_res
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(o_ptr, o_idx, x, n_dst)
        except Exception as exc:  # the baseline must never take the GPU line down
            res["cpu_baseline"] = {"value": None, "error": repr(exc)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
