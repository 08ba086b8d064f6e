#!/bin/bash
# rocprofv3 kernel statistics of the fused GAT forward/backward on C3 at each
# column-block count in BLOCKS (one profiled process per count).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${BLOCKS:-4 8}; do
  GAT_AB_BLOCKS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gatprof_$b -o run --output-format csv -- python3 scripts/gat_ab.py > gpurun_out/gatprof_$b.log 2>&1 || exit $?
  f=$(find gpurun_out/gatprof_$b -name "*kernel_stats.csv" | head -1)
  tail -5 gpurun_out/gatprof_$b.log; echo "== blocks $b"; cut -d, -f1-5 "$f" | head -12
done
