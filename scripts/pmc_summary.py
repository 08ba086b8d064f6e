#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_*) into profiles/pmc_traffic.json.

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE (KB) counts 128-B requests as 64 B for wide (16 B/lane) reads, so
it is doubled; WRITE_SIZE (KB) is exact for 16 B/lane stores.  Infinity-Cache
hits are included in both (they are L2 -> fabric requests).
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
vals = defaultdict(list)
for path in glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv")):
    keep = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "k_chunk_reduce" in name or "k_chunk_fixup" in name:
            k = "reduce" if "reduce" in name else "fixup"
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            keep.append(r)
    if keep:
        out = os.path.join(dst, "%s_%s.csv" % (tag, os.path.basename(os.path.dirname(path))))
        with open(out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(keep[0].keys()))
            w.writeheader()
            w.writerows(keep)
mean = {"%s/%s" % k: sum(v) / len(v) for k, v in vals.items()}
fetch = sum(mean.get("%s/FETCH_SIZE" % k, 0.0) for k in ("reduce", "fixup")) * 1024
write = sum(mean.get("%s/WRITE_SIZE" % k, 0.0) for k in ("reduce", "fixup")) * 1024
hit = mean.get("reduce/TCC_HIT_sum", 0.0)
miss = mean.get("reduce/TCC_MISS_sum", 0.0)
res = {
    "workload": "M1 copy_u_sum (scripts/tune_spmm.py --mode single), per launch pair k_chunk_reduce + k_chunk_fixup",
    "counters_mean_per_launch": mean,
    "fetch_bytes_raw": fetch,
    "write_bytes": write,
    "bytes_per_launch": 2 * fetch + write,
    "bytes_per_launch_uncorrected": fetch + write,
    "l2_hit_rate_reduce": hit / (hit + miss) if hit + miss else None,
    "note": "bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (gfx950 wide-read correction); includes Infinity-Cache hits",
}
json.dump(res, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
