#!/bin/bash
# Round 4: the 1-GPU bench line (PMC passes, configs children), the rocprofv3 kernel
# statistics of the same command, then the N = 2 rehearsal on this one GPU (gloo,
# --same-device, reduced sizes): per-rank roofline, c5 line, c4 speedup.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r04_bench.json | cut -c1-3000
[ $rc -eq 0 ] || { tail -20 gpurun_out/r04_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-update-all > gpurun_out/r04_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
export DGLMI_BENCH_TRACE=gpurun_out/r04_n2_trace
timeout -k 10 600 python -u bench.py --gpus 2 --same-device --dist-backend gloo \
  --edges-per-gpu 20000000 --scale 21 --c4-nodes 2000000 --c4-edges 40000000 \
  --c5-nodes 1000000 --c5-edges 16000000 --steps 5 --warmup 2 \
  > gpurun_out/r04_n2.json 2> gpurun_out/r04_n2.err
rc=$?; echo "n2 rc=$rc"; cat gpurun_out/r04_n2.json | cut -c1-4000; tail -5 gpurun_out/r04_n2.err
exit $rc
