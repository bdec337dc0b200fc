"""One GEMM configuration run repeatedly (for rocprofv3 --pmc / --kernel-trace passes).

python scripts/gemm_pmc.py M N K cfg [reps]   (cfg -1 = torch.matmul / hipBLASLt)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

M, N, K, cfg = (int(v) for v in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
for _ in range(reps):
    if cfg < 0:
        torch.matmul(x, w.t())
    else:
        G.linear(x, w, cfg=cfg, splits=1)
torch.cuda.synchronize()
print("done", M, N, K, cfg)
