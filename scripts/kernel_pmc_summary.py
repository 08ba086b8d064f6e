#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 counter passes (scripts/gpu_pmc_passes.sh): for each
kernel whose name contains one of the given substrings, every counter averaged over
its dispatches, plus derived fields -- fetch / write GB (FETCH_SIZE doubled for
gfx950's 16-B streaming reads, MI355X_MICROARCH.md), L2 hit rate, wait fraction.

usage: kernel_pmc_summary.py <prefix> <passes> <substr>[,<substr>...] [out.json]"""
import collections
import csv
import json
import sys


def main(prefix, passes, subs, out=None):
    res = collections.defaultdict(dict)
    for i in range(passes):
        rows = list(csv.DictReader(open("%s_%d/run_counter_collection.csv" % (prefix, i))))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            k = r["Kernel_Name"]
            if any(sb in k for sb in subs):
                name = k.replace("void dglmi::(anonymous namespace)::", "").split("(")[0]
                per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for (name, _), cs in per.items():
            for c, v in cs.items():
                agg[name][c].append(v)
        for name, cs in agg.items():
            for c, v in cs.items():
                res[name][c] = sum(v) / len(v)
                res[name]["dispatches_pass%d" % i] = len(v)
    for name, cs in res.items():
        if "FETCH_SIZE" in cs:
            cs["fetch_GB_raw"] = cs["FETCH_SIZE"] * 1024 / 1e9
            cs["fetch_GB_x2"] = 2 * cs["fetch_GB_raw"]
        if "WRITE_SIZE" in cs:
            cs["write_GB"] = cs["WRITE_SIZE"] * 1024 / 1e9
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            cs["l2_hit"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            cs["wait_frac"] = cs["SQ_WAIT_ANY"] / max(1.0, cs["SQ_WAVE_CYCLES"])
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3].split(","), sys.argv[4] if len(sys.argv) > 4 else None)
