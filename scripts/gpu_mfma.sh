#!/bin/bash
# MFMA utilisation of the bracketing GEMMs: one rocprofv3 --pmc pass per shape
# (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE), summarised by scripts/mfma_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in ${SHAPES:-c1 c2 c3 c5}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/mfma_$s -o run --output-format csv -- python3 scripts/mfma_probe.py --shape $s > gpurun_out/mfma_$s.log 2>&1
  rc=$?; echo "mfma $s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/mfma_summary.py gpurun_out gpurun_out ${TAG:-r01}
