#!/bin/bash
# N = 4 and N = 8 rehearsals of bench.py on ONE GPU (gloo ranks sharing cuda:0):
# checks the multi-rank code paths (partition, hybrid plan, exchanges, parity
# checks) at the full C4 size; gloo moves rows through host memory, so the
# times say nothing about RCCL / xGMI.  Then the corrected halo probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in ${NS:-4 8}; do
  DGLMI_BENCH_TRACE=gpurun_out/trace_n$N timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2955$N bench.py --gpus $N --dist-backend gloo --same-device --steps 2 --warmup 1 --edges-per-gpu 5000000 --scale 19 ${C4ARGS:-} > gpurun_out/rehearse_n$N.json 2> gpurun_out/rehearse_n$N.err
  rc=$?; echo "N=$N rc=$rc"; tail -c 1500 gpurun_out/rehearse_n$N.json; grep -v Gloo gpurun_out/rehearse_n$N.err | tail -4
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/halo_probe.py > gpurun_out/halo_probe.log 2>&1
rc=$?; echo "halo rc=$rc"; tail -3 gpurun_out/halo_probe.log
exit $rc
