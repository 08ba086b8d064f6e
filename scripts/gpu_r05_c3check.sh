set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_configs.py --configs c3 --steps 5 --warmup 2 > gpurun_out/r05_c3check.json 2> gpurun_out/r05_c3check.err
rc=$?; cat gpurun_out/r05_c3check.json | cut -c1-1500; tail -3 gpurun_out/r05_c3check.err; exit $rc
