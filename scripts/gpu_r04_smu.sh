#!/bin/bash
# Round 4: edge-softmax row pass, steps in flight per wave at H = 8 (4 in-tree, 8 in ab_u8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/softmax_rows_probe.py > gpurun_out/r04_smu4.json 2> gpurun_out/r04_smu4.err
rc=$?; echo "u4 rc=$rc"; cat gpurun_out/r04_smu4.json; [ $rc -eq 0 ] || exit $rc
DGL_LIBRARY_PATH=$PWD/ab_u8 timeout -k 10 300 python scripts/softmax_rows_probe.py > gpurun_out/r04_smu8.json 2> gpurun_out/r04_smu8.err
rc=$?; echo "u8 rc=$rc"; cat gpurun_out/r04_smu8.json
exit $rc
