#!/bin/bash
# Round 5: the unfused GATConv composition (C3) -- kernel / nn / generic / empty-row /
# int64 tests for the SDDMM and u_add_v gradient routes, the stage probe, and a kernel
# trace of module forward + backward steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_comp2}
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  ${TESTS:-tests/test_kernels_gpu.py tests/test_nn_gpu.py tests/test_generic_gpu.py tests/test_empty_rows_gpu.py \
  tests/test_int64_gpu.py tests/test_message_api_gpu.py tests/test_specialization_gpu.py} > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u scripts/gat_unfused_probe.py > gpurun_out/${T}_probe.json 2> gpurun_out/${T}_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/${T}_probe.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${T}_probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}prof -o run --output-format csv -- python3 scripts/gat_unfused_probe.py --module-only > gpurun_out/${T}prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the same module steps with attention dropout 0.6 (position space)
GAT_ATTN_DROP=0.6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}dropprof -o run --output-format csv -- python3 scripts/gat_unfused_probe.py --module-only > gpurun_out/${T}dropprof.log 2>&1
rc=$?; echo "rocprof (dropout) rc=$rc"; exit $rc
