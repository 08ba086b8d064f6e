#!/bin/bash
# Round 5 head: the whole GPU suite (timed), smoke, the headline bench with its PMC
# passes, CPU baseline and configs, then the rocprofv3 kernel statistics of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/r05_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc ($(( $(date +%s) - start )) s)"; tail -3 gpurun_out/r05_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r05_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/r05_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_benchprof -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-configs > gpurun_out/r05_benchprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
