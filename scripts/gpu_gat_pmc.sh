#!/bin/bash
# Kernel trace + PMC passes over the fused GAT kernels (scripts/gat_probe.py, C3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/gat_trace -o run --output-format csv -- python3 scripts/gat_probe.py > gpurun_out/gat_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/gat_trace.log; [ $rc -eq 0 ] || exit $rc
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/gat_pmc$i -o run --output-format csv -- python3 scripts/gat_probe.py --reps 2 > gpurun_out/gat_pmc$i.log 2>&1
  rc=$?; echo "pmc $i ($ctr) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/spmm_sq -o run --output-format csv -- python3 scripts/tune_spmm.py --mode single --steps 3 > gpurun_out/spmm_sq.log 2>&1
rc=$?; echo "spmm sq rc=$rc"; exit $rc
