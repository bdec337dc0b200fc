"""Seconds per diffusion step (UNet round trip incl. CFG batch doubling), random-init weights.

The reference logs "step i/n done, {dt}s" (cake-core/src/models/sd/sd.rs:506-507);
this measures the same quantity for a full-size UNet on one MI355X."""
import argparse
import json
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.models.sd.config import get_config  # noqa: E402
from cake_amd.models.sd.unet import UNet2DConditionModel  # noqa: E402
from cake_amd.models.sd.weights import random_component  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--version", default="v1-5")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--graph", action="store_true", help="replay the UNet step as one hipGraph")
    ap.add_argument("--denoise", action="store_true",
                    help="whole diffusion loop through SDUnit.denoise: device timestep, UNet, "
                         "CFG + scheduler update in one graph replay per step")
    ap.add_argument("--vae", action="store_true", help="time one VAE decode (batch 1) instead")
    ap.add_argument("--no-kv-cache", dest="kv_cache", action="store_false",
                    help="recompute the cross-attention k/v of the text context every step")
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    cfg = get_config(a.version)
    dev = torch.device("cuda:0")
    if a.vae:
        return bench_vae(a, cfg, dev, dt)
    if a.denoise:
        return bench_denoise(a, dev, dt)
    w = random_component("unet", cfg, dev, dt)
    unet = UNet2DConditionModel(cfg.unet)
    B = 2  # classifier-free guidance doubles the batch
    x = torch.randn(B, 4, cfg.height // 8, cfg.width // 8, device=dev, dtype=dt)
    ctx = torch.randn(B, 77, cfg.unet.cross_attention_dim, device=dev, dtype=dt)
    tbuf = torch.zeros((), device=dev)
    kv = {} if a.kv_cache else None  # cross-attn k/v of the (fixed) text context, as the pipeline
    with torch.no_grad():
        for _ in range(2):  # warmup: conv autotuning, packed weights, workspaces
            unet.forward(w, x, tbuf, ctx, kv)
        torch.cuda.synchronize()
        step = lambda: unet.forward(w, x, tbuf, ctx, kv)  # noqa: E731
        if a.graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                unet.forward(w, x, tbuf, ctx, kv)
            step = g.replay
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            tbuf.fill_(999 - i)
            step()
        torch.cuda.synchronize()
    dt_step = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"metric": "sd_unet_seconds_per_step", "version": a.version,
                      "resolution": f"{cfg.width}x{cfg.height}", "batch": B, "dtype": a.dtype,
                      "value": round(dt_step, 4), "unit": "s/step", "graph": a.graph,
                      "ctx_kv_cache": a.kv_cache,
                      "nhwc": os.environ.get("CAKE_SD_NHWC", "1") != "0"}))


def bench_vae(a, cfg, dev, dt):
    """VAE decode of one latent (incl. the head-dim-512 mid-block attention)."""
    from cake_amd.models.sd.vae import AutoencoderKL
    w = random_component("vae", cfg, dev, dt)
    vae = AutoencoderKL(cfg.vae)
    z = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, device=dev, dtype=dt)
    with torch.no_grad():
        for _ in range(2):
            vae.decode(w, z)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = max(1, a.steps)
        for _ in range(n):
            vae.decode(w, z)
        torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / n
    print(json.dumps({"metric": "sd_vae_decode_seconds", "version": a.version,
                      "resolution": f"{cfg.width}x{cfg.height}", "batch": 1, "dtype": a.dtype,
                      "value": round(dt_s, 4), "unit": "s"}))


def bench_denoise(a, dev, dt):
    from cake_amd.models.sd.bench import measure_denoise
    r = measure_denoise(a.version, a.steps, dt, dev)
    print(json.dumps({"metric": "sd_unet_seconds_per_step", "version": a.version,
                      "resolution": r["resolution"], "batch": 2, "dtype": a.dtype,
                      "value": round(r["seconds_per_step"], 4), "unit": "s/step", "graph": True,
                      "denoise": True, "scheduler": r["scheduler"], "steps": r["steps"],
                      "per_step_s": [round(x, 4) for x in r["per_step_s"]],
                      "nhwc": os.environ.get("CAKE_SD_NHWC", "1") != "0"}))


if __name__ == "__main__":
    main()
