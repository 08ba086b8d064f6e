#!/bin/bash
# Round 4: identity edge ids detected on dst-sorted graphs: tests, then the kinds probe
# on the dst-sorted C5 graph with the detection on and off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_streamed_edge_gpu.py tests/test_kernels_gpu.py tests/test_nn_gpu.py > gpurun_out/r04_sorted_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_sorted_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04_sorted_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/spmm_kinds_probe.py sorted > gpurun_out/r04_sorted_on.json 2> gpurun_out/r04_sorted_on.err
rc=$?; echo "on rc=$rc"; cat gpurun_out/r04_sorted_on.json
[ $rc -eq 0 ] || exit $rc
DGLMI_EID_IDENTITY=0 timeout -k 10 300 python scripts/spmm_kinds_probe.py sorted > gpurun_out/r04_sorted_off.json 2> gpurun_out/r04_sorted_off.err
rc=$?; echo "off rc=$rc"; cat gpurun_out/r04_sorted_off.json
exit $rc
