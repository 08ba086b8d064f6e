set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -k "special or blocked" -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_special.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_special.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u scripts/policy_probe.py --relabel > gpurun_out/policy_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -50 gpurun_out/policy_probe.log
exit $rc
