#!/bin/bash
# Round 4: the R-GCN GPU tests (fused kernels, C entries, module, reference ABI, C5
# full size), then the floor probe (copy_u_sum / u_mul_e_sum on the C5 graph vs the fused
# entries, pipelined forward A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_hack_capi_gpu.py tests/test_rgcn_gpu.py tests/test_rgcn_refabi_gpu.py tests/test_hack_oracle_gpu.py \
  "tests/test_configs_gpu.py::test_c5_rgcn_fused_route_full_size" > gpurun_out/r04_rgcn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_rgcn_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_rgcn_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/rgcn_floor_probe.py > gpurun_out/r04_floor2.json 2> gpurun_out/r04_floor2.err
rc=$?; echo "floor rc=$rc"; cat gpurun_out/r04_floor2.json
exit $rc
