#!/bin/bash
# Round 5: headline A/B -- the in-tree library (ids staged one batch ahead in
# k_chunk_reduce) against the previous head (dgl-hack_amd/variants/head), alternating,
# M1 copy_u_sum only; then the kernel suites that exercise k_chunk_reduce.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-pmc --no-cpu-baseline --no-c4 --no-configs --no-update-all"
for i in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export DGL_LIBRARY_PATH=$PWD/dgl-hack_amd/variants/head; else unset DGL_LIBRARY_PATH; fi
    timeout -k 10 300 python bench.py $B > gpurun_out/r05_ab_${v}_$i.json 2> gpurun_out/r05_ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(python3 -c "import json;d=json.loads(open('gpurun_out/r05_ab_${v}_$i.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))")"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_ab_${v}_$i.err; exit $rc; }
  done
done
unset DGL_LIBRARY_PATH
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_hub_rows_gpu.py tests/test_streamed_edge_gpu.py tests/test_generic_gpu.py tests/test_empty_rows_gpu.py tests/test_int64_gpu.py > gpurun_out/r05_ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_ab_tests.log
exit $rc
