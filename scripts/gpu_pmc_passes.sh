#!/bin/bash
# rocprofv3 counter passes, one counter group per run (the per-block limits of
# MI355X_MICROARCH.md): gpu_pmc_passes.sh <out-prefix> <python script> [args...].
# Writes <out-prefix>_<i>/run_counter_collection.csv; summarise with
# scripts/kernel_pmc_summary.py <out-prefix> 4 <kernel substrings>.
set -u
prefix=$1; shift
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d ${prefix}_$i -o run --output-format csv -- python3 "$@" > ${prefix}_$i.log 2>&1 || { echo "pmc pass $i ($c) failed"; exit 1; }
  i=$((i+1))
done
echo "pmc passes ok: $prefix"
