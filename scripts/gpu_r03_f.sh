#!/bin/bash
# Round 3: the hack entry points against the oracle restatement of the hack kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_hack_oracle_gpu.py > gpurun_out/r03f_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -20 gpurun_out/r03f_pytest.log
exit $rc
