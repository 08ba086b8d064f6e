#!/bin/bash
# Tuning + PMC session (separate rocprofv3 --pmc passes, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python scripts/tune_spmm.py --mode sweep --feats 16,64,128,256 > gpurun_out/tune.json 2> gpurun_out/tune.err
rc=$?; echo "tune rc=$rc"; cat gpurun_out/tune.json | head -80
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 scripts/tune_spmm.py --mode single --steps 3 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; tail -2 gpurun_out/pmc_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
