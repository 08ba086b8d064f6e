#!/bin/bash
# Round 4: the R-GCN reference-ABI / C5 parity tests, the fused GAT with the forward's
# slope aggregates (no destination-side backward walk), the DPP walk A/B on C5, and the
# C3 GAT timing both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=12 \
  tests/test_rgcn_refabi_gpu.py tests/test_hack_capi_gpu.py tests/test_hack_oracle_gpu.py \
  tests/test_rgcn_gpu.py tests/test_fused_gat_gpu.py tests/test_fused_gat_refabi_gpu.py \
  tests/test_nn_gpu.py tests/test_capture_gpu.py \
  "tests/test_configs_gpu.py::test_c5_rgcn_fused_route_full_size" \
  "tests/test_configs_gpu.py::test_c3_reddit_gat_fused_vs_unfused_and_sampled_fp64" > gpurun_out/r04d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 gpurun_out/r04d_pytest.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  DGLMI_PROBES=$v timeout -k 10 200 python -u scripts/c5_module_probe.py >> gpurun_out/r04d_rgcn_ab.jsonl 2>> gpurun_out/r04d_ab.err || { echo "rgcn probe $v failed"; tail -5 gpurun_out/r04d_ab.err; exit 1; }
  echo "rgcn probes=$v $(tail -1 gpurun_out/r04d_rgcn_ab.jsonl)"
done
for v in 1 0 1 0; do
  DGLMI_GAT_SLOPES=$v timeout -k 10 300 python -u scripts/bench_configs.py --configs c3 --steps 10 --warmup 3 >> gpurun_out/r04d_c3_ab.jsonl 2>> gpurun_out/r04d_ab.err || { echo "c3 $v failed"; tail -5 gpurun_out/r04d_ab.err; exit 1; }
  echo "gat slopes=$v $(tail -1 gpurun_out/r04d_c3_ab.jsonl)"
done
