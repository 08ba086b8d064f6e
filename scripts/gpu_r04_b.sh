#!/bin/bash
# Round 4: the N > 1 bench path rehearsed on one GPU (gloo, two ranks sharing it, reduced
# sizes): per-rank PMC roofline, the partitioned C5 R-GCN line, C4's speedup_vs_n1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export DGLMI_BENCH_TRACE=gpurun_out/r04b_trace
timeout -k 10 900 python -u bench.py --gpus 2 --same-device --dist-backend gloo \
  --edges-per-gpu 20000000 --scale 21 --c4-nodes 2000000 --c4-edges 40000000 \
  --c5-nodes 1000000 --c5-edges 16000000 --steps 5 --warmup 2 \
  > gpurun_out/r04b_n2.json 2> gpurun_out/r04b_n2.err
rc=$?; echo "n2 rc=$rc"; cat gpurun_out/r04b_n2.json; tail -20 gpurun_out/r04b_n2.err
exit $rc
