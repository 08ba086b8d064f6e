#!/bin/bash
# Bench with live PMC passes + rocprofv3 kernel stats of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${WITH_TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "special" -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_special.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_special.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -12 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-pmc --no-cpu-baseline --no-update-all --no-c4 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
exit $rc
