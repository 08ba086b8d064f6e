#!/bin/bash
# Round 5: row-owned softmax window / occupancy variants (probe builds under
# dgl-hack_amd/variants/, not shipped), then the N = 2 gloo rehearsal of bench.py with
# the round-5 N > 1 fields.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_softmax_owned_gpu.py tests/test_nn_gpu.py > gpurun_out/r05_sm2_tests.log 2>&1
rc=$?; echo "softmax tests rc=$rc"; tail -2 gpurun_out/r05_sm2_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r05_sm2_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/softmax_rows_probe.py > gpurun_out/r05_smvar_lds36.json 2> gpurun_out/r05_smvar_lds36.err
rc=$?; echo "lds36 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_smvar_lds36.err; exit $rc; }
for d in dgl-hack_amd/variants/*/; do
  v=$(basename $d)
  DGL_LIBRARY_PATH=$PWD/$d timeout -k 10 200 python scripts/softmax_rows_probe.py > gpurun_out/r05_smvar_$v.json 2> gpurun_out/r05_smvar_$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_smvar_$v.err; exit $rc; }
done
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_gat_dropout_gpu.py tests/test_fused_gat_gpu.py tests/test_rgcn_gpu.py tests/test_streamed_edge_gpu.py > gpurun_out/r05_drop_tests.log 2>&1
rc=$?; echo "drop tests rc=$rc"; tail -2 gpurun_out/r05_drop_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r05_drop_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/gat_dropout_probe.py > gpurun_out/r05_gatdrop.json 2> gpurun_out/r05_gatdrop.err
rc=$?; echo "gatdrop rc=$rc"; cat gpurun_out/r05_gatdrop.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_configs.py --configs c3 > gpurun_out/r05_c3.json 2> gpurun_out/r05_c3.err
rc=$?; echo "c3 rc=$rc"; cat gpurun_out/r05_c3.json; [ $rc -eq 0 ] || exit $rc
export DGLMI_BENCH_TRACE=gpurun_out/r05_n2_trace
timeout -k 10 600 python -u bench.py --gpus 2 --same-device --dist-backend gloo \
  --edges-per-gpu 20000000 --scale 21 --c4-nodes 2000000 --c4-edges 40000000 \
  --c5-nodes 1000000 --c5-edges 16000000 --steps 5 --warmup 2 \
  > gpurun_out/r05_n2.json 2> gpurun_out/r05_n2.err
rc=$?; echo "n2 rc=$rc"; cut -c1-300 gpurun_out/r05_n2.json; grep -iE "error|Traceback" gpurun_out/r05_n2.err | cut -c1-500 | head
exit $rc
