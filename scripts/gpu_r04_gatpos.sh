#!/bin/bash
# Round 4: GATConv composition in position space -- bit-identity tests, then the C3
# probe (stage medians, module with / without the position view).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_nn_gpu.py tests/test_gat_dropout_gpu.py tests/test_fused_gat_gpu.py > gpurun_out/r04_gatpos_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_gatpos_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_gatpos_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/gat_unfused_probe.py > gpurun_out/r04_gatpos.json 2> gpurun_out/r04_gatpos.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r04_gatpos.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_gatpos.err; exit $rc; }
exit $rc
