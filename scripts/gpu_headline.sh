#!/bin/bash
# Headline evidence: bench.py (N=1), rocprofv3 kernel stats of the same command,
# PMC traffic passes (separate runs, kernel-trace only) over the M1 copy_u_sum.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-update-all > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 scripts/tune_spmm.py --mode single --steps 3 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out gpurun_out ${TAG:-r01} > /dev/null
exit 0
