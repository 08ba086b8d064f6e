#!/bin/bash
# Round 4: the deferred-multiply / tie kernels: their tests, the C3 / C2 configs, and
# the per-kind probe on the C5 and M1 graphs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_streamed_edge_gpu.py tests/test_kernels_gpu.py tests/test_hub_rows_gpu.py \
  > gpurun_out/r04_kinds_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_kinds_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_kinds_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/spmm_kinds_probe.py > gpurun_out/r04_kinds_c5.json 2> gpurun_out/r04_kinds_c5.err
rc=$?; echo "kinds c5 rc=$rc"; cat gpurun_out/r04_kinds_c5.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/spmm_kinds_probe.py m1 > gpurun_out/r04_kinds_m1.json 2> gpurun_out/r04_kinds_m1.err
rc=$?; echo "kinds m1 rc=$rc"; cat gpurun_out/r04_kinds_m1.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_configs.py --configs c3,c2 > gpurun_out/r04_c3.json 2> gpurun_out/r04_c3.err
rc=$?; echo "configs rc=$rc"; cut -c1-500 gpurun_out/r04_c3.json
exit $rc
