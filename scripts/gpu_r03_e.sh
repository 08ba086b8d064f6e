#!/bin/bash
# Round 3 (re-entry): full GPU suite, smoke, bench and its kernel stats at the head,
# then whether two RCCL ranks can share the one GPU (for an N = 2 RCCL rehearsal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_r03_suite.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u scripts/rccl_same_device_probe.py > gpurun_out/r03_rccl_probe.log 2>&1
rc=$?; echo "rccl probe rc=$rc"; tail -5 gpurun_out/r03_rccl_probe.log
exit 0
