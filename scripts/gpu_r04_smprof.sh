#!/bin/bash
# Round 4: kernel statistics of the edge-softmax probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_smprof -o run --output-format csv -- python3 scripts/softmax_rows_probe.py > gpurun_out/r04_smprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/r04_smprof.log
exit $rc
