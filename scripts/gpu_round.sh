#!/bin/bash
# Full evidence session: GPU tests, smoke, bench, rocprofv3 kernel stats, PMC passes,
# secondary configs, C4 training example, 2-rank rehearsal.  Stops at the first
# crash/timeout (exit codes other than 0/1 from pytest, any non-zero elsewhere).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-update-all > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 scripts/tune_spmm.py --mode single --steps 3 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python scripts/bench_configs.py --configs c1,c2,c3,c5,sd,gemm > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python examples/dist_gcn.py > gpurun_out/dist_gcn.json 2> gpurun_out/dist_gcn.err
rc=$?; echo "dist_gcn rc=$rc"; cat gpurun_out/dist_gcn.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --edges-per-gpu 20000000 --scale 21 --dist-backend gloo --same-device > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; echo "bench n2 rehearsal rc=$rc"; cat gpurun_out/bench_n2.json
exit $rc
