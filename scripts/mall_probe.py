"""Does a weight matrix read just before a GEMV (plain loads, allocating in the 256 MB
Infinity Cache / MALL) make the GEMV's non-temporal weight stream faster?  o_proj shape
of Llama-3-8B (4096 x 4096 bf16, 32 MiB) and gate/up (28672 x 4096, 224 MiB)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402


def timed(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        pre()
        torch.cuda.synchronize()
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


flush = torch.empty(1 << 29, dtype=torch.uint8, device="cuda")  # 512 MiB
for N in (4096, 14336 * 2):
    W = torch.randn(N, 4096, device="cuda").to(torch.bfloat16)
    x = torch.randn(4096, device="cuda").to(torch.bfloat16)
    out = torch.zeros(N, device="cuda")
    sink = torch.zeros(1, device="cuda")
    for mode in ("cold", "mall"):
        def pre():
            flush.fill_(1)  # evict
            if mode == "mall":
                sink.copy_(W.amax())  # plain-load pass over W
        us = timed(lambda: K.gemv(x, W, out, accumulate=False))
        print(json.dumps({"N": N, "K": 4096, "mode": mode, "gemv_us": round(us, 2),
                          "TBps": round(N * 4096 * 2 / us / 1e6, 2)}), flush=True)
