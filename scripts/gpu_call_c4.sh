#!/bin/bash
# Partition tests, then bench at N = 1 (M1 + C4) and a 2-rank gloo rehearsal on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_partition_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_partition.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_partition.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-pmc --no-cpu-baseline --steps 10 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_n1.json; tail -5 gpurun_out/bench_n1.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --same-device --steps 3 --warmup 1 --edges-per-gpu 20000000 --scale 21 --no-exchange > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "bench2 rc=$rc"; cat gpurun_out/bench_n2.json; tail -5 gpurun_out/bench_n2.err
exit $rc
