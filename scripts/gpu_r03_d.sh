#!/bin/bash
# Round 3: fused R-GCN layer-1 kernels: tests, C5 probe, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_hack_capi_gpu.py tests/test_configs_gpu.py tests/test_rgcn_gpu.py -k "rgcn or c5" > gpurun_out/r03d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03d_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rgcn_capi_probe.py > gpurun_out/r03_rgcn_capi3.json 2> gpurun_out/r03_rgcn_capi3.err
rc=$?; echo "rgcn probe rc=$rc"; cat gpurun_out/r03_rgcn_capi3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_rgcn_trace3 -o run --output-format csv -- python3 scripts/rgcn_capi_probe.py --capi-only --fused > gpurun_out/r03_rgcn_trace3.log 2>&1
rc=$?; echo "rgcn trace rc=$rc"
exit $rc
