#!/bin/bash
# Round 5: tall-skinny fp32 MFMA GEMM probe (C2 projection shape) against torch.matmul
# (hipBLASLt) on the same shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/gemm_ts_probe > gpurun_out/r05_gemm_ts.json 2>&1
rc=$?; cat gpurun_out/r05_gemm_ts.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 - <<'PY' >> gpurun_out/r05_gemm_ts.json
import json, torch as th
x = th.rand(169343, 128, device="cuda") * 2 - 1
w = th.rand(128, 128, device="cuda") * 2 - 1
for name, f in (("torch_x_wT", lambda: x @ w.t()), ("torch_x_w", lambda: x @ w)):
    f(); th.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); th.cuda.synchronize(); ts.append(a.elapsed_time(b))
    print(json.dumps({"kernel": name, "best_ms": min(ts[1:])}))
PY
rc=$?; tail -2 gpurun_out/r05_gemm_ts.json; exit $rc
