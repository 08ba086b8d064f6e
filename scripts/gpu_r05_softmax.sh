#!/bin/bash
# Round 5: row-owned edge softmax -- its tests and the mapped u_mul_e fix, the softmax
# and edge-softmax suites, then the probe (graph / view chunked / view owned) and a
# rocprofv3 kernel trace of the probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_softmax_owned_gpu.py tests/test_streamed_edge_gpu.py tests/test_nn_gpu.py tests/test_kernels_gpu.py tests/test_hub_rows_gpu.py tests/test_int64_gpu.py tests/test_fused_gat_gpu.py > gpurun_out/r05_sm4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_sm4_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r05_sm4_tests.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/softmax_rows_probe.py > gpurun_out/r05_sm4_probe.json 2> gpurun_out/r05_sm4_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r05_sm4_probe.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05_sm4_probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_sm4prof -o run --output-format csv -- python3 scripts/softmax_rows_probe.py > gpurun_out/r05_sm4prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
