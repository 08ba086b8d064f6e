set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GAT_ATTN_DROP=0.6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_dropprof -o run --output-format csv -- python3 scripts/gat_unfused_probe.py --module-only > gpurun_out/r05_dropprof.log 2>&1
echo "rc=$?"
