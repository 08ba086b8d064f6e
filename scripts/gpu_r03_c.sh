#!/bin/bash
# Round 3: tall-skinny GEMMs of the R-GCN C entries (tests + C5 probe + kernel
# stats), fused-GAT chunk-size sweep on the probe build (C3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_hack_capi_gpu.py tests/test_configs_gpu.py -k "rgcn or c5" > gpurun_out/r03c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03c_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rgcn_capi_probe.py > gpurun_out/r03_rgcn_capi2.json 2> gpurun_out/r03_rgcn_capi2.err
rc=$?; echo "rgcn probe rc=$rc"; cat gpurun_out/r03_rgcn_capi2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_rgcn_trace2 -o run --output-format csv -- python3 scripts/rgcn_capi_probe.py --capi-only --prepared > gpurun_out/r03_rgcn_trace2.log 2>&1
rc=$?; echo "rgcn trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune_gat.py > gpurun_out/r03_tune_gat.json 2> gpurun_out/r03_tune_gat.err
rc=$?; echo "tune gat rc=$rc"; cat gpurun_out/r03_tune_gat.json; tail -3 gpurun_out/r03_tune_gat.err
exit $rc
