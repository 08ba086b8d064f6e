#!/bin/bash
# Round 4: fused R-GCN walk with DPP row broadcasts (shipped build) vs the round-3
# ds_bpermute walk (probe build), C5 module fwd / fwd+bwd, A B A; then the parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 0 1; do
  DGLMI_PROBES=$v timeout -k 10 200 python -u scripts/c5_module_probe.py >> gpurun_out/r04c_ab.jsonl 2>> gpurun_out/r04c_ab.err || { echo "probe $v failed"; tail -5 gpurun_out/r04c_ab.err; exit 1; }
  echo "probes=$v $(tail -1 gpurun_out/r04c_ab.jsonl)"
done
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_hack_capi_gpu.py tests/test_hack_oracle_gpu.py tests/test_rgcn_gpu.py tests/test_rgcn_refabi_gpu.py > gpurun_out/r04c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r04c_pytest.log
exit $rc
