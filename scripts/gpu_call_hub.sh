#!/bin/bash
# Segmented fixups: hub-row parity tests, the hub probe, the headline kernel
# time, then the full GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hub_rows_gpu.py tests/test_fused_gat_gpu.py tests/test_empty_rows_gpu.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_hub.log 2>&1
rc=$?; echo "hub tests rc=$rc"; tail -15 gpurun_out/pytest_hub.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/hub_probe.py > gpurun_out/hub_probe.json 2> gpurun_out/hub_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/hub_probe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --no-c4 --no-update-all > gpurun_out/bq.json 2>/dev/null
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bq.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_suite.sh
