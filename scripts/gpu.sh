#!/bin/bash
# One parameterised launcher for the GPU box (gpurun), replacing the per-round one-offs.
#   scripts/gpu.sh TAG tests [pytest args / test files...]   GPU tests (-x), log gpurun_out/TAG_tests.log
#   scripts/gpu.sh TAG suite                                  the whole GPU suite (no -x) + smoke
#   scripts/gpu.sh TAG configs c2,c3,c5 [extra args]          scripts/bench_configs.py -> gpurun_out/TAG_configs.json
#   scripts/gpu.sh TAG bench [bench.py args]                  bench.py -> gpurun_out/TAG_bench.json
#   scripts/gpu.sh TAG stats [bench.py args]                  rocprofv3 --kernel-trace --stats over bench.py
#   scripts/gpu.sh TAG py SCRIPT [args]                       any probe script -> gpurun_out/TAG_py.log
# Every GPU step runs under its own time limit; a failing step ends the call (chain calls with &&).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; mode=$2; shift 2
out=gpurun_out/${tag}
case "$mode" in
  tests)
    timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
      -m gpu "$@" > ${out}_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 ${out}_tests.log
    [ $rc -eq 0 ] || grep -E "Error|assert|FAILED|Traceback" ${out}_tests.log | head -30
    exit $rc ;;
  suite)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 \
      --timeout-method thread -rf > ${out}_suite.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -15 ${out}_suite.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${out}_smoke.log 2>&1
    rc2=$?; echo "smoke rc=$rc2"; tail -2 ${out}_smoke.log
    [ $rc -eq 0 ] && exit $rc2; exit $rc ;;
  configs)
    list=$1; shift
    timeout -k 10 600 python -u scripts/bench_configs.py --configs "$list" "$@" > ${out}_configs.json 2> ${out}_configs.err
    rc=$?; echo "configs rc=$rc"; cut -c1-1500 ${out}_configs.json; [ $rc -eq 0 ] || tail -20 ${out}_configs.err
    exit $rc ;;
  bench)
    timeout -k 10 900 python -u bench.py "$@" > ${out}_bench.json 2> ${out}_bench.err
    rc=$?; echo "bench rc=$rc"; cut -c1-3000 ${out}_bench.json; [ $rc -eq 0 ] || tail -20 ${out}_bench.err
    exit $rc ;;
  stats)
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d ${out}_prof -o run -- python3 bench.py "$@" \
      > ${out}_stats.log 2>&1
    rc=$?; echo "stats rc=$rc"; tail -3 ${out}_stats.log
    find ${out}_prof -name '*kernel_stats.csv' | head -3
    exit $rc ;;
  py)
    script=$1; shift
    timeout -k 10 900 python -u "$script" "$@" > ${out}_py.log 2>&1
    rc=$?; echo "py rc=$rc"; tail -40 ${out}_py.log
    exit $rc ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
