#!/bin/bash
# round 5: where the first library-GEMM call's time goes (handle / library init vs a new
# kernel's code object vs a new plan)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python - <<'PY'
import time, torch
from cake_amd.ops import gemm as G
def t(M, N, K, tag):
    x = torch.randn(M, K, device="cuda").bfloat16(); w = torch.randn(N, K, device="cuda").bfloat16()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    G.linear(x, w, cfg=G.LIB); torch.cuda.synchronize()
    print(f"{tag}: M={M} N={N} K={K} {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
t(8, 64, 64, "first call, tiny shape")
t(8, 64, 64, "same tiny shape again")
t(2048, 6144, 4096, "first big shape")
t(2048, 6144, 4096, "big shape again")
t(2048, 4096, 14336, "second big shape")
t(1000, 6144, 4096, "new M of a seen shape")
PY
