#!/bin/bash
# Round 5: the MFMA projection kernel -- its tests, the modules that project (nn, configs,
# examples, capture, R-GCN), then the C2 / C3 / C5 configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_nn_gpu.py tests/test_capture_gpu.py tests/test_rgcn_gpu.py tests/test_examples_gpu.py \
  tests/test_configs_gpu.py tests/test_conv_zoo_gpu.py tests/test_hetero_gpu.py > gpurun_out/r05_proj_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_proj_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r05_proj_tests.log | head -30; exit $rc; }
timeout -k 10 400 python -u scripts/bench_configs.py --configs c2,c3,c5 --steps 10 --warmup 3 > gpurun_out/r05_proj_configs.json 2> gpurun_out/r05_proj_configs.err
rc=$?; echo "configs rc=$rc"; cut -c1-700 gpurun_out/r05_proj_configs.json; exit $rc
