"""Flash attention forward: the 16-row kernel (impl 1) vs the 32x32x16 swapped-QKᵀ kernel
(impl 2) on the SD / SDXL / Llama-prefill shapes.  One JSON line per shape."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402

# name, B, H, Hkv, N, M, D, causal
SHAPES = [
    ("sdxl.self.64x64", 2, 10, 10, 4096, 4096, 64, False),
    ("sdxl.self.32x32", 2, 20, 20, 1024, 1024, 64, False),
    ("sdxl.cross.64x64", 2, 10, 10, 4096, 77, 64, False),
    ("sd15.self.64x64", 2, 8, 8, 4096, 4096, 40, False),
    ("sd15.self.32x32", 2, 8, 8, 1024, 1024, 80, False),
    ("llama8b.prefill.2048", 1, 32, 8, 2048, 2048, 128, True),
    ("llama8b.prefill.512", 1, 32, 8, 512, 512, 128, True),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    for name, B, H, Hkv, N, M, D, causal in SHAPES:
        q = torch.randn(B, N, H, D, device=dev).to(dt).transpose(1, 2)
        k = torch.randn(B, M, Hkv, D, device=dev).to(dt).transpose(1, 2)
        v = torch.randn(B, M, Hkv, D, device=dev).to(dt).transpose(1, 2)
        o = torch.empty(B, N, H, D, device=dev, dtype=dt).transpose(1, 2)
        flops = 4.0 * B * H * N * M * D * (0.5 if causal else 1.0)
        rec = {"shape": name}
        outs = {}
        for impl in (1, 2):
            K.flash_set_impl(impl)
            t = timeit(lambda: K.flash_attn(q, k, v, o, 1 / math.sqrt(D), causal))
            outs[impl] = o.clone()
            rec[f"impl{impl}_us"] = round(t, 1)
            rec[f"impl{impl}_tflops"] = round(flops / t / 1e6, 1)
        rec["max_diff"] = round((outs[1].float() - outs[2].float()).abs().max().item(), 4)
        print(json.dumps(rec), flush=True)
    K.flash_set_impl(2)


if __name__ == "__main__":
    main()
