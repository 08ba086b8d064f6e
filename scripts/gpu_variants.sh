#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python scripts/tune_spmm.py --mode sweep --feats 64 --chunks ${CHUNKS:-256,512} --variants ${VARIANTS:-0,1,2,3,4,7} --rounds 3 > gpurun_out/variants.json 2> gpurun_out/variants.err
rc=$?; echo "variants rc=$rc"
python - <<'PY'
import json
d=json.load(open('gpurun_out/variants.json'))
for k,v in sorted(d.items(), key=lambda kv: kv[1]['ms']): print(k, round(v['ms'],4), round(v['min_ms'],4), round(v['alg_GBps']))
PY
exit $rc
