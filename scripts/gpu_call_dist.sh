#!/bin/bash
# Distributed-path GPU tests, then the C4 training example on one GPU and as a
# 2-rank gloo rehearsal (hybrid and pull exchanges).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_partition_gpu.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/dist_gcn.jsonl
for ex in hybrid pull; do
  timeout -k 10 200 python -u examples/dist_gcn.py --epochs 3 --warmup 1 --exchange $ex >> gpurun_out/dist_gcn.jsonl 2> gpurun_out/dist_gcn.err || exit $?
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 examples/dist_gcn.py --same-device --dist-backend gloo --nodes 1000000 --edges 20000000 --epochs 2 --warmup 1 --exchange $ex >> gpurun_out/dist_gcn.jsonl 2>> gpurun_out/dist_gcn.err || exit $?
done
cat gpurun_out/dist_gcn.jsonl
