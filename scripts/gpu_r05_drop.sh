#!/bin/bash
# Round 5: attention dropout without the per-edge hash path -- dropout / GAT tests, the
# dropout probe and the C3 config, then the counter passes of the dropout probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_gat_dropout_gpu.py tests/test_fused_gat_gpu.py tests/test_nn_gpu.py > gpurun_out/r05_drop2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_drop2_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r05_drop2_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/gat_dropout_probe.py > gpurun_out/r05_gatdrop2.json 2> gpurun_out/r05_gatdrop2.err
rc=$?; echo "gatdrop rc=$rc"; cat gpurun_out/r05_gatdrop2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_configs.py --configs c3 > gpurun_out/r05_c3b.json 2> gpurun_out/r05_c3b.err
rc=$?; echo "c3 rc=$rc"; cat gpurun_out/r05_c3b.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_gatdrop2_prof -o run --output-format csv -- python3 scripts/gat_dropout_probe.py > gpurun_out/r05_gatdrop2_prof.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_passes.sh gpurun_out/r05_gatpmc2 scripts/gat_dropout_probe.py || exit 1
python3 scripts/kernel_pmc_summary.py gpurun_out/r05_gatpmc2 4 k_gat_ gpurun_out/r05_gatpmc2.json > /dev/null || exit 1
echo done
