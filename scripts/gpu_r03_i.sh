#!/bin/bash
# Round 3: edge-position GAT backward restricted to unblocked walks: A/B on C3 and
# the GAT / capture / refabi / hack-oracle tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GAT_AB_POS="1 0" timeout -k 10 300 python -u scripts/gat_ab.py > gpurun_out/r03i_gat_ab.json 2> gpurun_out/r03i_gat_ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r03i_gat_ab.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03i_gat_ab.err; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_fused_gat_gpu.py tests/test_fused_gat_refabi_gpu.py tests/test_hack_oracle_gpu.py tests/test_nn_gpu.py tests/test_capture_gpu.py tests/test_int64_gpu.py > gpurun_out/r03i_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03i_pytest.log
exit $rc
