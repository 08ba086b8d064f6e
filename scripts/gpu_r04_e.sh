#!/bin/bash
# Round 4: parity tests (R-GCN reference ABI, 16-row fused R-GCN kernel and the 32-row
# one, fused GAT with slope aggregates, full-size C5 / C3), then A/B timings: the fused
# R-GCN kernels (round-3 walk = probe build / DPP walk on 32-row tiles / 16-row tiles,
# 16 waves per CU) on the C5 module, and the GAT backward with the forward's slope
# aggregates vs the edge-position path vs the destination walk on C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 850 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=12 \
  tests/test_rgcn_refabi_gpu.py tests/test_hack_capi_gpu.py tests/test_hack_oracle_gpu.py \
  tests/test_rgcn_gpu.py tests/test_fused_gat_gpu.py tests/test_fused_gat_refabi_gpu.py \
  tests/test_nn_gpu.py tests/test_capture_gpu.py \
  "tests/test_configs_gpu.py::test_c5_rgcn_fused_route_full_size" \
  "tests/test_configs_gpu.py::test_c3_reddit_gat_fused_vs_unfused_and_sampled_fp64" > gpurun_out/r04e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 gpurun_out/r04e_pytest.log
[ $rc -eq 0 ] || exit $rc
for v in r3 t32 t16 t16 t32 r3; do
  case $v in r3) P=1; T=32;; t32) P=0; T=32;; t16) P=0; T=16;; esac
  DGLMI_PROBES=$P DGLMI_RGCN_TILE=$T timeout -k 10 200 python -u scripts/c5_module_probe.py > gpurun_out/r04e_one.json 2>> gpurun_out/r04e_ab.err || { echo "rgcn probe $v failed"; tail -5 gpurun_out/r04e_ab.err; exit 1; }
  echo "{\"variant\": \"$v\", \"res\": $(cat gpurun_out/r04e_one.json)}" | tee -a gpurun_out/r04e_rgcn_ab.jsonl
done
GAT_AB_BLOCKS="auto 1" GAT_AB_POS="slopes 1 0" timeout -k 10 300 python -u scripts/gat_ab.py > gpurun_out/r04e_gat_ab.json 2>> gpurun_out/r04e_ab.err
rc=$?; echo "gat ab rc=$rc"; cat gpurun_out/r04e_gat_ab.json
exit $rc
