#!/bin/bash
# Full GPU suite (with the slowest tests listed), smoke, the headline bench and the
# rocprofv3 kernel statistics of the same bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=30 > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r03_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-update-all > gpurun_out/r03_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
