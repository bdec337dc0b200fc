"""Causal flash attention (Llama prefill shapes) with and without q-tile pairing:
µs per call and TFLOP/s (causal FLOPs), graph of back-to-back launches."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    for (H, Hkv, D, N) in [(32, 8, 128, 512), (32, 8, 128, 1024), (32, 8, 128, 2048),
                           (32, 8, 128, 4096), (64, 8, 128, 1024), (64, 8, 128, 2048),
                           (32, 8, 128, 8192), (12, 12, 64, 77)]:
        q = torch.randn(1, N, H, D, device=dev).to(dt).transpose(1, 2)
        k = torch.randn(1, N, Hkv, D, device=dev).to(dt).transpose(1, 2)
        v = torch.randn(1, N, Hkv, D, device=dev).to(dt).transpose(1, 2)
        out = torch.empty(1, N, H, D, device=dev, dtype=dt).transpose(1, 2)
        rec = {"H": H, "D": D, "N": N}
        flops = 4.0 * N * N * D * H / 2
        for name, pm, nw in (("unpaired", 0, 0), ("paired", 1, 0), ("nw2", 0, 2),
                             ("nw2_paired", 1, 2), ("auto", 512, 0)):
            K.flash_set_pair_min(pm)
            K.kernels().cake_flash_set_nw(nw)
            K.flash_attn(q, k, v, out, 1 / math.sqrt(D), True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    K.flash_attn(q, k, v, out, 1 / math.sqrt(D), True)
            g.replay()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                g.replay()
                b.record()
                b.synchronize()
                best = min(best, a.elapsed_time(b) * 1e3 / 10)
            rec[f"{name}_us"] = round(best, 1)
            rec[f"{name}_tflops"] = round(flops / best / 1e6, 1)
        K.flash_set_pair_min(512)
        K.kernels().cake_flash_set_nw(0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
