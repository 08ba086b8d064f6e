#!/bin/bash
# Targeted GPU session: selected test files, then (optional) secondary configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_quick.log
ok $rc || exit $rc
if [ -n "${CONFIGS:-}" ]; then
  timeout -k 10 900 python scripts/bench_configs.py --configs $CONFIGS > gpurun_out/configs.json 2> gpurun_out/configs.err
  rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.json; tail -5 gpurun_out/configs.err
fi
exit 0
