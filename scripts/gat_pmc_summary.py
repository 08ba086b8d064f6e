#!/usr/bin/env python3
"""Summarise the fused-GAT rocprofv3 passes of scripts/gpu_gat_pmc.sh (C3:
232,965 nodes, 114.6 M edges, 8 heads x 8) into one JSON per kernel: calls,
average duration (kernel trace), and per WALK (one call = num_col_blocks
launches) the bytes past L2 (FETCH_SIZE x 2, the gfx950 wide-read correction of
MI355X_MICROARCH.md section HBM, + WRITE_SIZE), the L2 hit rate and the L2
request count, beside the line-request model of DESIGN.md section 4.3.

usage: gat_pmc_summary.py [gpurun_out] [out.json] [col_blocks]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r03_gat_pmc_blocked.json"
blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 8
E = 114_615_892
H, D = 8, 8
TRACE_CALLS = 6
KERNELS = ("k_gat_fwd<", "k_gat_fwd_fixup", "k_gat_merge", "k_gat_bwd_dst", "k_gat_bwd_src",
           "k_gat_bwd_fixup")


def kname(name):
    for k in KERNELS:
        if k in name:
            return k.rstrip("<")
    return None


vals = defaultdict(list)
for path in glob.glob(os.path.join(src, "gat_pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
dur = {}
for r in csv.DictReader(open(os.path.join(src, "gat_trace", "run_kernel_stats.csv"))):
    k = kname(r["Name"])
    if k:
        dur[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6}

# line requests per edge of each walk: forward ft[u] 256 B = 2
# lines + el[u]; destination-side backward the same 3; source-side backward
# dO[v] 2 lines + the packed {er, m, 1/l, delta}[v] line
model_lines = {"k_gat_fwd": 3, "k_gat_bwd_dst": 3, "k_gat_bwd_src": 3}
alg_bytes = {"k_gat_fwd": E * (4 * H * D + 4 * H + 8),
             "k_gat_bwd_dst": E * (4 * H * D + 4 * H + 8),
             "k_gat_bwd_src": E * (4 * H * D + 16 * H + 8)}
res = {"workload": "C3 Reddit-size Chung-Lu graph, 232965 nodes, %d edges, GAT 8 heads x 8, "
                   "column blocks B = %d (one launch per block; a walk = B launches)" % (E, blocks),
       "source": "scripts/gpu_gat_pmc.sh over scripts/gat_probe.py (EXTRA_PMC=WRITE_SIZE), "
                 "one counter group per rocprofv3 pass",
       "fetch_correction": "FETCH_SIZE x 2 (gfx950 counts 128-B wide reads as 64 B)",
       "kernels": {}}
for k in sorted({k for k, _ in vals}):
    mean = {c: sum(v) / len(v) for (kk, c), v in vals.items() if kk == k}
    per_launch_read = mean.get("FETCH_SIZE", 0.0) * 1024 * 2
    per_launch_write = mean.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = mean.get("TCC_HIT_sum", 0.0), mean.get("TCC_MISS_sum", 0.0)
    # launches per walk from the trace: gat_probe.py makes 1 + 5 calls of each
    # direction (the fixups run once per block launch, k_gat_bwd_fixup for both
    # backward walks)
    walk = dur[k]["calls"] / TRACE_CALLS if k in dur else blocks
    if k == "k_gat_bwd_fixup":
        walk /= 2
    d = {"launches_per_walk": walk,
         "bytes_past_l2_per_walk": (per_launch_read + per_launch_write) * walk,
         "read_bytes_per_walk": per_launch_read * walk,
         "write_bytes_per_walk": per_launch_write * walk,
         "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
         "l2_requests_per_walk": (hit + miss) * walk,
         "valu_insts_per_walk": mean.get("SQ_INSTS_VALU", 0.0) * walk}
    if k in dur:
        d.update(dur[k])
        d["ms_per_walk"] = dur[k]["avg_ms"] * walk
        if k == "k_gat_bwd_fixup":
            d["note"] = "per backward walk (the fixup follows both walks)"
        d["fabric_GBps"] = d["bytes_past_l2_per_walk"] / (d["ms_per_walk"] * 1e-3) / 1e9
    if k in model_lines:
        d["model_line_requests_per_walk"] = model_lines[k] * E
        d["l2_requests_per_edge"] = d["l2_requests_per_walk"] / E
        d["alg_bytes_per_walk"] = alg_bytes[k]
        d["traffic_over_alg"] = d["bytes_past_l2_per_walk"] / alg_bytes[k]
    res["kernels"][k] = d
os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
json.dump(res, open(dst, "w"), indent=1)
for k, d in res["kernels"].items():
    print("%-16s %s" % (k, {kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in d.items()}))
