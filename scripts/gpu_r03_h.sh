#!/bin/bash
# Round 3: fused GAT backward without the destination-side walk (edge positions):
# C3 A/B (auto blocks / unblocked x edge-position / destination walk), a kernel trace
# of the new backward, then the fused GAT parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GAT_AB_POS="1 0" timeout -k 10 300 python -u scripts/gat_ab.py > gpurun_out/r03h_gat_ab.json 2> gpurun_out/r03h_gat_ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r03h_gat_ab.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03h_gat_ab.err; exit $rc; }
GAT_AB_BLOCKS=auto timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03h_trace -o run --output-format csv -- python3 scripts/gat_ab.py > gpurun_out/r03h_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_fused_gat_gpu.py tests/test_fused_gat_refabi_gpu.py tests/test_hack_oracle_gpu.py tests/test_nn_gpu.py tests/test_hub_rows_gpu.py tests/test_capture_gpu.py > gpurun_out/r03h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03h_pytest.log
exit $rc
