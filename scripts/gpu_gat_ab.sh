#!/bin/bash
# Fused GAT A/B on one box: each library under abtest/ (VARIANTS), then the
# fused GAT parity tests on the library named by TESTLIB (default: in-tree).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/gat_ab.jsonl
for v in ${VARIANTS:-in-tree}; do
  lib=$PWD/abtest/$v; [ "$v" = in-tree ] && lib=$PWD/dgl-hack_amd/dgl/_lib
  DGL_LIBRARY_PATH=$lib timeout -k 10 240 python -u scripts/gat_ab.py --save gpurun_out/gat_$v.pt >> gpurun_out/gat_ab.jsonl 2> gpurun_out/gat_ab_$v.err || exit $?
done
cat gpurun_out/gat_ab.jsonl
if [ -n "${TESTLIB:-}" ]; then export DGL_LIBRARY_PATH=$PWD/abtest/$TESTLIB; fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_fused_gat_gpu.py tests/test_nn_gpu.py} -m gpu > gpurun_out/pytest_gat.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gat.log; rm -f gpurun_out/*.pt; exit $rc
