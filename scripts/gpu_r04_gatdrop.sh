#!/bin/bash
# Round 4: kernel trace of the fused GAT with and without attention dropout (C3 size).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_gatdrop -o run --output-format csv -- python3 scripts/gat_dropout_probe.py > gpurun_out/r04_gatdrop.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/r04_gatdrop.log
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r04_gatdrop/run_kernel_trace.csv")))
d = collections.defaultdict(list)
for r in rows:
    if "k_gat" in r["Kernel_Name"]:
        d[r["Kernel_Name"].split("(")[0][-60:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print(k, len(v), [round(x, 3) for x in v[:4]], "...", [round(x, 3) for x in v[-4:]])
PY
