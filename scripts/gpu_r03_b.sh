#!/bin/bash
# Round 3: GPU tests of the reference-order fused GAT entries, the prepared R-GCN
# state and the touched kernels; C5 R-GCN C-entry probe (+ rocprofv3 kernel
# stats of the prepared entries); M1 hot/cold split probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_fused_gat_refabi_gpu.py tests/test_hack_capi_gpu.py tests/test_fused_gat_gpu.py \
  tests/test_generic_gpu.py tests/test_partition_gpu.py tests/test_host_cpu.py > gpurun_out/r03b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rgcn_capi_probe.py > gpurun_out/r03_rgcn_capi.json 2> gpurun_out/r03_rgcn_capi.err
rc=$?; echo "rgcn probe rc=$rc"; cat gpurun_out/r03_rgcn_capi.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_rgcn_trace -o run --output-format csv -- python3 scripts/rgcn_capi_probe.py --capi-only --prepared > gpurun_out/r03_rgcn_trace.log 2>&1
rc=$?; echo "rgcn trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/hotsplit_probe.py > gpurun_out/r03_hotsplit.json 2> gpurun_out/r03_hotsplit.err
rc=$?; echo "hotsplit rc=$rc"; cat gpurun_out/r03_hotsplit.json; tail -3 gpurun_out/r03_hotsplit.err
exit $rc
