#!/bin/bash
# Round 5: the N = 2 rehearsal on one GPU (gloo, --same-device, reduced sizes): the
# aggregated roofline, per-rank SpMM / exchange fields of c4 and c5, the c4 model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --same-device --dist-backend gloo \
  --edges-per-gpu 20000000 --scale 21 --c4-nodes 2000000 --c4-edges 40000000 \
  --c5-nodes 1000000 --c5-edges 16000000 --steps 5 --warmup 2 \
  > gpurun_out/r05_n2b.json 2> gpurun_out/r05_n2b.err
rc=$?; echo "n2 rc=$rc"; cut -c1-600 gpurun_out/r05_n2b.json; grep -E "error|Error" gpurun_out/r05_n2b.err | cut -c1-2000
exit $rc
