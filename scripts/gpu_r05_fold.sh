#!/bin/bash
# Round 5: the folded R-GCN backward (DGLMI_RGCN_FOLD=1) -- small graphs first (parity
# against the G_t + GEMM backward for R = 1, 2, 4), then C5 size with R = 2 (no register
# spills) and R = 4 (spilled), timing both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 1 2 4; do
  timeout -k 10 120 python scripts/rgcn_fold_probe.py $R 200000 3200000 > gpurun_out/r05_fold_small_$R.json 2> gpurun_out/r05_fold_small_$R.err
  rc=$?; echo "small R=$R rc=$rc $(cat gpurun_out/r05_fold_small_$R.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_fold_small_$R.err; exit $rc; }
done
for R in 2 4; do
  timeout -k 10 240 python scripts/rgcn_fold_probe.py $R > gpurun_out/r05_fold_c5_$R.json 2> gpurun_out/r05_fold_c5_$R.err
  rc=$?; echo "C5 R=$R rc=$rc $(cat gpurun_out/r05_fold_c5_$R.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_fold_c5_$R.err; exit $rc; }
done
