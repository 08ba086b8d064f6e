#!/usr/bin/env python3
"""Summarise scripts/gpu_rgcn_pmc.sh's counter passes per kernel (means over the
dispatches of each kernel; FETCH_SIZE in KB as rocprofv3 reports it)."""
import collections
import csv
import json
import sys


def main(root="gpurun_out", out=None):
    res = collections.defaultdict(dict)
    for i in range(4):
        rows = list(csv.DictReader(open("%s/rgcn_pmc_%d/run_counter_collection.csv" % (root, i))))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            k = r["Kernel_Name"]
            if "k_rgcn_fused" in k or "k_gemm_tn" in k:
                name = k.replace("void dglmi::(anonymous namespace)::", "").split("(")[0]
                per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for (name, _), cs in per.items():
            for c, v in cs.items():
                agg[name][c].append(v)
        for name, cs in agg.items():
            for c, v in cs.items():
                res[name][c] = sum(v) / len(v)
                res[name]["dispatches"] = len(v)
    for name, cs in res.items():
        simd_cycles = cs["GRBM_GUI_ACTIVE"] / 8 * 1024  # 8 XCDs; 256 CUs x 4 SIMDs
        cs["mfma_util"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        cs["wait_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
        cs["l2_hit"] = cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        cs["fetch_GB_raw"] = cs["FETCH_SIZE"] * 1024 / 1e9
        cs["write_GB"] = cs["WRITE_SIZE"] * 1024 / 1e9
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
