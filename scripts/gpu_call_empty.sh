#!/bin/bash
# Empty-row runs: the new parity tests, the locality probe (degree-sorted /
# BFS-ordered M1, long empty runs), then the full GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_empty_rows_gpu.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_empty.log 2>&1
rc=$?; echo "empty-rows tests rc=$rc"; tail -15 gpurun_out/pytest_empty.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/locality_probe.py > gpurun_out/locality_probe.json 2> gpurun_out/locality_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/locality_probe.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_suite.sh
