#!/bin/bash
# round 5: register-resident prefill RMSNorm: tests, then per-call time vs the loop kernel
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rmsnorm" > gpurun_out/r5_an.log 2>&1
rc=$?; tail -2 gpurun_out/r5_an.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 120 python - <<'PY'
import torch, json
from cake_amd.ops import hip as K, _lib
lib = _lib.kernels()
for T, H in ((2048, 4096), (4096, 4096), (2048, 8192), (512, 4096)):
    x = torch.randn(T, H, device="cuda"); w = torch.randn(H, device="cuda").bfloat16()
    out = torch.empty(T, H, device="cuda", dtype=torch.bfloat16)
    res = {}
    for _ in range(3):
        for reg in (1, 0):
            lib.cake_rmsnorm_set_reg(reg)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    K.rmsnorm(x, w, 1e-5, out)
            g.replay(); torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); g.replay(); b.record(); b.synchronize()
            res[reg] = min(res.get(reg, 1e9), a.elapsed_time(b) / 20 * 1e3)
    lib.cake_rmsnorm_set_reg(1)
    print(json.dumps({"T": T, "H": H, "reg_us": round(res[1], 2), "loop_us": round(res[0], 2),
                      "reg_TBps": round(T * H * 6 / res[1] / 1e6, 2)}))
PY
