#!/bin/bash
# Head check after the side-line guard: the default N = 1 bench, then an N = 2
# gloo rehearsal on one GPU (C4 scaled to 1 M / 20 M) through the guarded side lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?; echo "bench N=1 rc=$rc"; tail -c 600 gpurun_out/bench_n1.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 2 --dist-backend gloo --same-device --steps 2 --warmup 1 --edges-per-gpu 5000000 --scale 19 --c4-nodes 1000000 --c4-edges 20000000 > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err
rc=$?; echo "N=2 rc=$rc"; tail -c 1200 gpurun_out/rehearse_n2.json; exit $rc
