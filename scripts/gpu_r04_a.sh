#!/bin/bash
# Round 4: R-GCN entries in the reference's argument lists (etypes in the graph),
# DGLMIRgcnRefreshNorm, the full-size C5 parity test, and the verified C5 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread --durations=15 \
  tests/test_rgcn_refabi_gpu.py tests/test_hack_capi_gpu.py tests/test_hack_oracle_gpu.py \
  tests/test_rgcn_gpu.py tests/test_capture_gpu.py tests/test_distributed_gpu.py \
  "tests/test_configs_gpu.py::test_c5_rgcn_fused_route_full_size" > gpurun_out/r04a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r04a_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_configs.py --configs c5 --steps 10 --warmup 3 > gpurun_out/r04a_c5.json 2> gpurun_out/r04a_c5.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/r04a_c5.json; tail -3 gpurun_out/r04a_c5.err
exit $rc
