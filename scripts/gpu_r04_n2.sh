#!/bin/bash
# Round 4: the N = 2 rehearsal on one GPU (gloo, --same-device, reduced sizes): per-rank
# roofline, the partitioned c5 line, c4 speedup; and the graph-determinism probe first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/lp_determinism_probe.py > gpurun_out/r04_lpdet.json 2> gpurun_out/r04_lpdet.err
rc=$?; echo "lpdet rc=$rc"; cat gpurun_out/r04_lpdet.json
[ $rc -eq 0 ] || exit $rc
export DGLMI_BENCH_TRACE=gpurun_out/r04_n2_trace
timeout -k 10 600 python -u bench.py --gpus 2 --same-device --dist-backend gloo \
  --edges-per-gpu 20000000 --scale 21 --c4-nodes 2000000 --c4-edges 40000000 \
  --c5-nodes 1000000 --c5-edges 16000000 --steps 5 --warmup 2 \
  > gpurun_out/r04_n2.json 2> gpurun_out/r04_n2.err
rc=$?; echo "n2 rc=$rc"; cut -c1-600 gpurun_out/r04_n2.json; grep -E "^c5|error" gpurun_out/r04_n2.err | cut -c1-2000
exit $rc
