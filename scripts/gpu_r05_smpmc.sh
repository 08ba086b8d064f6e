#!/bin/bash
# Round 5: counters of the edge-softmax routes after the chunked row pass became the
# owned-walk form (k_sm_rows_v): graph (edge-id walk), view chunked, view owned, H = 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_pmc_passes.sh gpurun_out/r05_smpmc2 scripts/softmax_rows_probe.py --pmc || exit 1
python3 scripts/kernel_pmc_summary.py gpurun_out/r05_smpmc2 4 k_sm_ gpurun_out/r05_smpmc2.json > /dev/null || exit 1
echo done
