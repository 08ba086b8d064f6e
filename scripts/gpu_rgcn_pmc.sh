#!/bin/bash
# rocprofv3 counter passes over scripts/c5_module_probe.py (the C5 RelGraphConv on the
# fused layer-1 kernels), one pass per counter group; summarised by
# scripts/rgcn_pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d gpurun_out/rgcn_pmc_$i -o run --output-format csv -- python3 scripts/c5_module_probe.py > gpurun_out/rgcn_pmc_$i.log 2>&1 || { echo "pmc pass $i ($c) failed"; exit 1; }
  i=$((i+1))
done
echo "pmc passes ok"
