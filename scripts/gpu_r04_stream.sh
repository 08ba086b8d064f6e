#!/bin/bash
# Round 4: streamed constant edge operands (dgl.backend._StreamedEdgeReduce): the new
# tests, the kernel / generic / R-GCN suites that route through binary_reduce, then the
# C5-graph floor probe (u_mul_e_sum now streams the norm).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_streamed_edge_gpu.py tests/test_kernels_gpu.py tests/test_generic_gpu.py tests/test_rgcn_gpu.py \
  tests/test_nn_gpu.py tests/test_conv_zoo_gpu.py > gpurun_out/r04_stream_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_stream_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_stream_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/rgcn_floor_probe.py > gpurun_out/r04_floor3.json 2> gpurun_out/r04_floor3.err
rc=$?; echo "floor rc=$rc"; cat gpurun_out/r04_floor3.json
exit $rc
