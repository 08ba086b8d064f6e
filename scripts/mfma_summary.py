#!/usr/bin/env python3
"""Summarise the MFMA PMC passes of scripts/mfma_probe.py into
profiles/<tag>_mfma_util.json.

Per probe run (gpurun_out/mfma_<shape>/run_counter_collection.csv plus the probe's
JSON line in gpurun_out/mfma_<shape>.log): the dispatches that issued MFMA work
(SQ_VALU_MFMA_BUSY_CYCLES > 0) are the GEMMs.  For each op (forward, input
gradient, weight gradient):

* mfma_util = sum(SQ_VALU_MFMA_BUSY_CYCLES) / sum(GRBM_GUI_ACTIVE / 8 * 1024):
  busy SIMD-cycles over the cycles the GEMM kernels ran (GRBM_GUI_ACTIVE is summed
  over the 8 XCDs, MI355X_MICROARCH.md "DVFS give-back") times the 1024 SIMDs;
* counter_flops = busy cycles * 64 (an fp32 MFMA, 32x32x2 or 16x16x4, does 64 FLOP
  per SIMD-cycle), against the algorithmic 2*M*K*N per GEMM -- the check that the
  counter means what the formula assumes;
* tflops = algorithmic FLOPs / (end - start) of those dispatches, against the
  157.3 TFLOP/s dense fp32 matrix peak.

The weight-gradient op is the split-K product of dgl.backend.weight_grad: its
batched GEMM (and the remainder addmm) is counted here, the small slice sum (no
MFMA) is not.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles"
tag = sys.argv[3] if len(sys.argv) > 3 else "r01"
PEAK = 157.3
res = {"method": __doc__.strip().splitlines()[0], "peak_fp32_matrix_tflops": PEAK, "shapes": {}}
for log in sorted(glob.glob(os.path.join(src, "mfma_*.log"))):
    shape = os.path.basename(log)[len("mfma_"):-len(".log")]
    meta = None
    for line in open(log):
        line = line.strip()
        if line.startswith("{"):
            meta = json.loads(line)
    path = os.path.join(src, "mfma_" + shape, "run_counter_collection.csv")
    if meta is None or not os.path.exists(path):
        continue
    disp = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    gemms = [disp[k] for k in sorted(disp) if disp[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) > 0]
    reps, ops = meta["reps"], meta["ops"]
    entry = {"m": meta["m"], "k": meta["k"], "n": meta["n"], "mfma_dispatches": len(gemms)}
    # forward and input gradient are one GEMM each; the split-K weight gradient is a
    # batched GEMM plus, when the slices leave a remainder of rows, one addmm
    if len(gemms) >= 3 * reps:
        groups = [(ops[0], gemms[:reps]), (ops[1], gemms[reps:2 * reps]),
                  (ops[2], gemms[2 * reps:])]
    else:
        groups = [("all", gemms)]
    for op, ds in groups:
        busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in ds)
        cyc = sum(d["GRBM_GUI_ACTIVE"] / 8.0 for d in ds)
        ns = sum(d["ns"] for d in ds)
        n_gemm = reps if op != "all" else reps * len(ops)
        flops = meta["flops_per_gemm"] * n_gemm
        entry[op] = {
            "kernels": sorted({d["name"][:80] for d in ds}),
            "mfma_util": busy / (cyc * 1024) if cyc else None,
            "counter_flops_over_alg": busy * 64 / flops if flops else None,
            "ms_per_gemm": ns / 1e6 / n_gemm,
            "tflops": flops / (ns * 1e-9) / 1e12 if ns else None,
            "frac_of_peak": flops / (ns * 1e-9) / 1e12 / PEAK if ns else None,
        }
    res["shapes"][shape] = entry
out = os.path.join(dst, "%s_mfma_util.json" % tag)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
