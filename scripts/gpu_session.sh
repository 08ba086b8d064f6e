#!/bin/bash
# Incremental evidence session: selected GPU tests, bench N=1, 2-rank rehearsal
# (gloo, one GPU) incl. the with-exchange line, rocprof of the GAT config.
# Stops at the first crash/timeout.  TESTS / STEPS env override.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,bench,n2,gatprof}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if has bench; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if has n2; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --edges-per-gpu 20000000 --scale 21 --dist-backend gloo --same-device > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
  rc=$?; echo "bench n2 rehearsal rc=$rc"; cat gpurun_out/bench_n2.json; tail -5 gpurun_out/bench_n2.err
  [ $rc -eq 0 ] || exit $rc
fi
if has gatprof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gat -o run --output-format csv -- python3 scripts/bench_configs.py --configs c3 --steps 5 --warmup 2 > gpurun_out/prof_gat.log 2>&1
  rc=$?; echo "gat rocprof rc=$rc"; tail -3 gpurun_out/prof_gat.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
