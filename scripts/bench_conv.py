"""conv2d.hip vs MIOpen (torch, channels_last) on the Stable Diffusion conv shapes.

Prints one JSON line per shape: our time with the planner's choice, the best
(cfg, splits) of a sweep, and MIOpen's time on the same NHWC data.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402

# (name, N, H, W, IC, OC, k, stride, up)
SHAPES = [
    ("sd15.64.320", 2, 64, 64, 320, 320, 3, 1, False),
    ("sd15.32.640", 2, 32, 32, 640, 640, 3, 1, False),
    ("sd15.16.1280", 2, 16, 16, 1280, 1280, 3, 1, False),
    ("sd15.8.1280", 2, 8, 8, 1280, 1280, 3, 1, False),
    ("sd15.8.2560-1280", 2, 8, 8, 2560, 1280, 3, 1, False),
    ("sd15.64.960-320", 2, 64, 64, 960, 320, 3, 1, False),
    ("sd15.64.640-320.1x1", 2, 64, 64, 640, 320, 1, 1, False),
    ("sd15.down.64-32.320", 2, 64, 64, 320, 320, 3, 2, False),
    ("sd15.up.32-64.640", 2, 32, 32, 640, 640, 3, 1, True),
    ("sdxl.128.320", 2, 128, 128, 320, 320, 3, 1, False),
    ("sdxl.64.640", 2, 64, 64, 640, 640, 3, 1, False),
    ("sdxl.32.1280", 2, 32, 32, 1280, 1280, 3, 1, False),
    ("vae.512.128", 1, 512, 512, 128, 128, 3, 1, False),
    ("vae.256.256", 1, 256, 256, 256, 256, 3, 1, False),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--dtype", default="f16")
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    for name, N, H, W, IC, OC, k, stride, up in SHAPES:
        x = torch.randn(N, H, W, IC, device=dev).to(dt)
        w = (torch.randn(OC, IC, k, k, device=dev) / (IC * k * k) ** 0.5).to(dt)
        b = torch.randn(OC, device=dev).to(dt)
        wp = w.permute(0, 2, 3, 1).contiguous()
        pad = k // 2
        VH, VW = H << up, W << up
        OH, OW = (VH + 2 * pad - k) // stride + 1, (VW + 2 * pad - k) // stride + 1
        flops = 2.0 * N * OH * OW * OC * IC * k * k
        xn = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last

        def lib():
            xi = F.interpolate(xn, scale_factor=2.0, mode="nearest") if up else xn
            return F.conv2d(xi, w.to(memory_format=torch.channels_last), b, stride=stride, padding=pad)
        t_lib = timeit(lib, a.iters)
        t_ours = timeit(lambda: K.conv2d_nhwc(x, wp, b, stride=stride, pad=pad, up=up), a.iters)
        ref = lib().permute(0, 2, 3, 1).float()
        err = (K.conv2d_nhwc(x, wp, b, stride=stride, pad=pad, up=up).float() - ref).abs().max().item()
        P, ks = N * OH * OW, k * k * IC // 64
        rec = {"shape": name, "plan": K.conv_plan(P, OC, ks), "ours_us": round(t_ours, 1),
               "miopen_us": round(t_lib, 1), "ours_tflops": round(flops / t_ours / 1e6, 1),
               "miopen_tflops": round(flops / t_lib / 1e6, 1), "max_abs_err": round(err, 4)}
        if a.sweep:
            best = None
            for cfg in range(14):
                if cfg >= 8 and stride != 1:
                    continue
                for sp in ((1,) if cfg >= 8 else (1, 2, 4, 8)):
                    t = timeit(lambda: K.conv2d_nhwc(x, wp, b, stride=stride, pad=pad, up=up,
                                                     cfg=cfg, splits=sp), a.iters)
                    if best is None or t < best[0]:
                        best = (round(t, 1), cfg, sp)
            rec["best"] = best
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
