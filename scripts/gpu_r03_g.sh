#!/bin/bash
# Round 3: 64-bit graphs (int64 offsets / edge ids), then the kernel regression tests
# and the headline bench (the 64-bit reads must not cost the int32 path anything).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread --durations=10 \
  tests/test_int64_gpu.py > gpurun_out/r03g_int64.log 2>&1
rc=$?; echo "int64 rc=$rc"; tail -25 gpurun_out/r03g_int64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_generic_gpu.py tests/test_hub_rows_gpu.py tests/test_empty_rows_gpu.py > gpurun_out/r03g_kernels.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -3 gpurun_out/r03g_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/r03g_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
exit $rc
