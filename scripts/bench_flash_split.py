"""Non-causal flash attention at the Stable Diffusion UNet shapes (self and cross
attention, CFG batch 2): µs per call (incl. the merge launch) for each key-split count of
the v2 kernel (0 = automatic pick, 1 = no split, 2, 4).
Graph of 10 back-to-back launches, best of 5 replays; one JSON line per shape."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402

SHAPES = [  # name, B, H, N (queries), M (keys), D
    ("sdxl.l1.self", 2, 10, 4096, 4096, 64), ("sdxl.l1.cross", 2, 10, 4096, 77, 64),
    ("sdxl.l2.self", 2, 20, 1024, 1024, 64), ("sdxl.l2.cross", 2, 20, 1024, 77, 64),
    ("sd15.l0.self", 2, 8, 4096, 4096, 40), ("sd15.l0.cross", 2, 8, 4096, 77, 40),
    ("sd15.l1.self", 2, 8, 1024, 1024, 80), ("sd15.l1.cross", 2, 8, 1024, 77, 80),
]


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    for name, B, H, N, M, D in SHAPES:
        q = torch.randn(B, N, H, D, device=dev).to(dt).transpose(1, 2)
        k = torch.randn(B, M, H, D, device=dev).to(dt).transpose(1, 2)
        v = torch.randn(B, M, H, D, device=dev).to(dt).transpose(1, 2)
        out = torch.empty(B, N, H, D, device=dev, dtype=dt).transpose(1, 2)
        ref = None
        rec = {"shape": name, "B": B, "H": H, "N": N, "M": M, "D": D}
        flops = 4.0 * B * H * N * M * D
        for nw in (0, 1, 2, 4):
            K.flash_set_ksplit(nw)
            K.flash_attn(q, k, v, out, 1 / math.sqrt(D))
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            rec[f"ks{nw}_maxdiff"] = round(float((out.float() - ref).abs().max()), 4)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    K.flash_attn(q, k, v, out, 1 / math.sqrt(D))
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
            rec[f"ks{nw}_us"] = round(best, 1)
            rec[f"ks{nw}_tflops"] = round(flops / best / 1e6, 1)
        K.flash_set_ksplit(0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
