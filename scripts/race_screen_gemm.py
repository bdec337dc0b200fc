"""Race screen for a GEMM tile config: many launches at several shapes, each compared
bit-for-bit against the first launch and against an f32 reference (one process)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 14
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
bad = 0
for (M, N, K) in [(4096, 4096, 4096), (2048, 6144, 4096), (1000, 1300, 2112), (8192, 8192, 1024)]:
    torch.manual_seed(M + N + K)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    ref = (x.float() @ w.float().t())
    first = G.linear(x, w, cfg=cfg, splits=1).clone()
    err = (first.float() - ref).abs().max().item()
    same = 0
    for _ in range(reps):
        y = G.linear(x, w, cfg=cfg, splits=1)
        same += int(torch.equal(y, first))
    torch.cuda.synchronize()
    ok = same == reps and err < 0.05 * max(1.0, ref.abs().max().item())
    bad += int(not ok)
    print(f"cfg {cfg} {M}x{N}x{K}: max|err| {err:.4f}, identical {same}/{reps} {'OK' if ok else 'MISMATCH'}",
          flush=True)
sys.exit(1 if bad else 0)
