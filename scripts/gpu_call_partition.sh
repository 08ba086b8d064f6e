#!/bin/bash
# Partitioner: GPU tests, then the C4 quality / cost probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_partition_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_partition.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_partition.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u scripts/partition_probe.py ${PROBE_ARGS:-} > gpurun_out/partition_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -40 gpurun_out/partition_probe.log
exit $rc
