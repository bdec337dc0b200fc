"""Isolated timing of one GEMM shape with a given dtype / epilogue (rocprofv3 kernel-trace
run): python scripts/gemm_epi_probe.py M N K cfg dtype epi [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

M, N, K, cfg = (int(v) for v in sys.argv[1:5])
dt = {"bf16": torch.bfloat16, "f16": torch.float16}[sys.argv[5]]
epi = sys.argv[6]
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(dt)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(dt) * 0.05
b = (torch.rand(N, device="cuda") * 2 - 1).to(dt)
r = (torch.rand(M, N, device="cuda") * 2 - 1).to(dt)
out = torch.empty(M, N, device="cuda", dtype=dt)
for _ in range(reps):
    if epi == "add16":
        G.linear(x, w, b, epi="add16", out=out, resid=r, cfg=cfg, splits=1)
    else:
        G.linear(x, w, out=out, cfg=cfg, splits=1)
torch.cuda.synchronize()
print("done", M, N, K, cfg, sys.argv[5], epi)
