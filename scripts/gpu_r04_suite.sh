#!/bin/bash
# Round 4: the full GPU suite (slowest 60 listed) and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=60 > gpurun_out/r04_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r04_pytest_gpu.log | tail -2
[ $rc -eq 0 ] || { tail -40 gpurun_out/r04_pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04_smoke.log
exit $rc
