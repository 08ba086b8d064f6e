#!/bin/bash
# Round 4: C3 GATConv composition stages on the position view, kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gat_unfused_probe.py > gpurun_out/r04_gatpos2.json 2> gpurun_out/r04_gatpos2.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r04_gatpos2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_gatpos2.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_gatpos_prof -o run --output-format csv -- python3 scripts/gat_unfused_probe.py --kernels > gpurun_out/r04_gatpos_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
