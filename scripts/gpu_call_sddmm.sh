#!/bin/bash
# Narrow SDDMM timings, then FETCH_SIZE / request-size / hit-rate passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/sddmm_probe.jsonl
timeout -k 10 120 python -u scripts/sddmm_probe.py >> gpurun_out/sddmm_probe.jsonl 2> gpurun_out/sddmm_probe.err || exit $?
cat gpurun_out/sddmm_probe.jsonl
for pv in 0; do
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/sddmm_pmc_v${pv}_$tag -o run --output-format csv -- python3 scripts/sddmm_probe.py --once --heads 8 > /dev/null 2>&1 || { echo "pmc $c failed"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, json
out = {}
for f in glob.glob("gpurun_out/sddmm_pmc_*/**/*counter_collection.csv", recursive=True):
    tag = f.split("/")[1]
    for r in csv.DictReader(open(f)):
        if "sddmm" in r["Kernel_Name"]:
            out.setdefault(tag, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(json.dumps({t: {c: sum(v) / len(v) for c, v in d.items()} for t, d in out.items()}))
json.dump(out, open("gpurun_out/sddmm_pmc.json", "w"))
PY
