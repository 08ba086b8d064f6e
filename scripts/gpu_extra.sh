#!/bin/bash
# Secondary configs + multi-rank rehearsal of bench.py (2 ranks on one GPU, gloo).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_configs.py --configs ${CONFIGS:-c1,c2,c3} > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.json; tail -5 gpurun_out/configs.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --edges-per-gpu 20000000 --scale 21 --dist-backend gloo --same-device > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "bench n2 rehearsal rc=$rc"; cat gpurun_out/bench_n2.json; tail -5 gpurun_out/bench_n2.err
exit $rc
