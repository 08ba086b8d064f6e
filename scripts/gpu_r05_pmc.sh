#!/bin/bash
# Round 5: counters of the edge-softmax routes (chunked vs row-owned, C3 view H = 8) and
# of the fused GAT with / without attention dropout; kernel trace of the dropout probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_gatdrop_prof -o run --output-format csv -- python3 scripts/gat_dropout_probe.py > gpurun_out/r05_gatdrop_prof.log 2>&1
rc=$?; echo "gatdrop trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_passes.sh gpurun_out/r05_smpmc scripts/softmax_rows_probe.py --pmc || exit 1
python3 scripts/kernel_pmc_summary.py gpurun_out/r05_smpmc 4 k_sm_ gpurun_out/r05_smpmc.json > /dev/null || exit 1
bash scripts/gpu_pmc_passes.sh gpurun_out/r05_gatpmc scripts/gat_dropout_probe.py || exit 1
python3 scripts/kernel_pmc_summary.py gpurun_out/r05_gatpmc 4 k_gat_ gpurun_out/r05_gatpmc.json > /dev/null || exit 1
echo done
