#!/bin/bash
# Full evidence session: GPU tests, smoke, headline bench + rocprofv3 kernel stats +
# PMC traffic, MFMA utilisation of the GEMMs, fused-GAT PMC, secondary configs,
# the partitioned training examples and a 2-rank rehearsal of bench.py.  Stops at
# the first failure (pytest failures included: rc 1 means a failed test).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_headline.sh || exit $?
bash scripts/gpu_mfma.sh > gpurun_out/mfma.out 2>&1 || exit $?
bash scripts/gpu_gat_pmc.sh > gpurun_out/gat_pmc.out 2>&1 || exit $?
timeout -k 10 900 python scripts/bench_configs.py --configs c1,c2,c3,c5,c5h,sd,gemm > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python examples/dist_gcn.py > gpurun_out/dist_gcn.json 2> gpurun_out/dist_gcn.err
rc=$?; echo "dist_gcn rc=$rc"; cat gpurun_out/dist_gcn.json
[ $rc -eq 0 ] || exit $rc
for m in gat rgcn; do
  timeout -k 10 600 python examples/dist_train.py --model $m > gpurun_out/dist_train_$m.json 2> gpurun_out/dist_train_$m.err
  rc=$?; echo "dist_train $m rc=$rc"; cat gpurun_out/dist_train_$m.json
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --edges-per-gpu 20000000 --scale 21 --dist-backend gloo --same-device > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "bench n2 rehearsal rc=$rc"; cat gpurun_out/bench_n2.json
exit $rc
