#!/bin/bash
# Round 3: (1) bench.py --gpus 2 with no torchrun (the script starts its own two
# ranks; gloo, both on cuda:0, small knobs); (2) fused GAT kernels on C3 under
# rocprofv3: kernel trace + PMC passes (SQ, TCC hit/miss, FETCH_SIZE, WRITE_SIZE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --same-device --steps 3 --warmup 1 \
  --edges-per-gpu 10000000 --scale 20 --c4-nodes 1000000 --c4-edges 20000000 \
  > gpurun_out/launch_n2.json 2> gpurun_out/launch_n2.err
rc=$?; echo "launch n2 rc=$rc"; tail -c 1200 gpurun_out/launch_n2.json; grep -v Gloo gpurun_out/launch_n2.err | tail -6
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_GAT:-0}" = 1 ] && exit 0
EXTRA_PMC="WRITE_SIZE" bash scripts/gpu_gat_pmc.sh
