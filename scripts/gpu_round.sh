#!/bin/bash
# Full evidence session: GPU tests, smoke, bench, rocprofv3 kernel stats, PMC passes,
# secondary configs.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 scripts/tune_spmm.py --mode single --steps 3 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python scripts/bench_configs.py > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.json
exit 0
