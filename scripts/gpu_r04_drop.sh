#!/bin/bash
# Round 4: attention dropout inside the fused GAT kernels: its tests, the GAT suites,
# then the C3 config (with the dropout lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_gat_dropout_gpu.py tests/test_fused_gat_gpu.py tests/test_fused_gat_refabi_gpu.py \
  tests/test_hack_oracle_gpu.py tests/test_nn_gpu.py tests/test_examples_gpu.py > gpurun_out/r04_drop_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_drop_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_drop_tests.log | head -20; exit $rc; }
timeout -k 10 400 python scripts/bench_configs.py --configs c3 > gpurun_out/r04_c3drop.json 2> gpurun_out/r04_c3drop.err
rc=$?; echo "c3 rc=$rc"; cat gpurun_out/r04_c3drop.json
exit $rc
