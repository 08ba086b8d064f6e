#!/bin/bash
# Round 4: lane-per-head edge-softmax row kernel -- softmax / GAT tests, then the
# softmax probe, then the C3 composition probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_nn_gpu.py tests/test_kernels_gpu.py tests/test_hub_rows_gpu.py tests/test_int64_gpu.py tests/test_fused_gat_gpu.py > gpurun_out/r04_smrows_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_smrows_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_smrows_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/softmax_rows_probe.py > gpurun_out/r04_smrows_new.json 2> gpurun_out/r04_smrows_new.err
rc=$?; echo "new rc=$rc"; cat gpurun_out/r04_smrows_new.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_smrows_new.err; exit $rc; }
timeout -k 10 300 python scripts/gat_unfused_probe.py > gpurun_out/r04_gatpos3.json 2> gpurun_out/r04_gatpos3.err
rc=$?; echo "gat rc=$rc"; cat gpurun_out/r04_gatpos3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_smprof2 -o run --output-format csv -- python3 scripts/softmax_rows_probe.py > gpurun_out/r04_smprof2.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
