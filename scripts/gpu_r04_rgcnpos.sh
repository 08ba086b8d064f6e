#!/bin/bash
# Round 4: R-GCN prepared walks as position walks (null edge ids -> staged weights):
# the R-GCN GPU tests, then the C-entry probe against the previous library (A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_hack_capi_gpu.py tests/test_rgcn_gpu.py tests/test_rgcn_refabi_gpu.py \
  "tests/test_configs_gpu.py::test_c5_rgcn_fused_route_full_size" > gpurun_out/r04_rgcnpos_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_rgcnpos_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_rgcnpos_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/rgcn_capi_probe.py > gpurun_out/r04_capi_new.json 2> gpurun_out/r04_capi_new.err
rc=$?; echo "new rc=$rc"; cat gpurun_out/r04_capi_new.json; [ $rc -eq 0 ] || exit $rc
DGL_LIBRARY_PATH=$PWD/ab_old timeout -k 10 300 python scripts/rgcn_capi_probe.py > gpurun_out/r04_capi_old.json 2> gpurun_out/r04_capi_old.err
rc=$?; echo "old rc=$rc"; cat gpurun_out/r04_capi_old.json
exit $rc
