"""Stable Diffusion seconds per diffusion step (the reference's second metric:
"step i/n done, {dt}s", cake-core/src/models/sd/sd.rs:464-513, 506-507), measured on a
random-init full-size UNet: classifier-free guidance doubles the batch, and every step
is one hipGraph replay of time embedding -> UNet -> CFG combine + scheduler update
(SDUnit.denoise).  Used by bench.py (``sd`` sub-record) and scripts/bench_sd.py."""
from __future__ import annotations

import time

import torch


def measure_denoise(version: str = "xl", steps: int = 8, dtype=torch.float16,
                    device="cuda:0") -> dict:
    from .config import get_config
    from .schedulers import build_scheduler
    from .shardable import SDUnit
    from .weights import random_component
    dev = torch.device(device)
    cfg = get_config(version)
    w = random_component("unet", cfg, dev, dtype)
    unit = SDUnit("unet", cfg, w, dev, dtype)
    ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim, device=dev, dtype=dtype)
    sched = build_scheduler(cfg.scheduler, steps + 2)
    ts = sched.timesteps()
    lat = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, device=dev) * sched.init_noise_sigma
    with torch.no_grad():
        unit.denoise(lat, ctx, sched, ts, 7.5, True, 1)  # step 0 eager (autotune), capture
        unit.denoise(lat, ctx, sched, ts, 7.5, True, 3)  # replay-only warm pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, per = unit.denoise(lat, ctx, sched, ts, 7.5, True, 2)
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / len(ts)
    out = {"seconds_per_step": round(wall, 5), "version": version,
           "resolution": f"{cfg.width}x{cfg.height}", "batch": 2,
           "dtype": "f16" if dtype == torch.float16 else "bf16",
           "scheduler": cfg.scheduler.kind, "steps": len(ts),
           "per_step_s": [round(x, 5) for x in per]}
    del unit, w
    torch.cuda.empty_cache()
    return out


def measure_native(version: str = "xl", steps: int = 8, dtype: str = "f16",
                   device: int = 0) -> dict:
    """The same metric on the native SD engine (csrc/engine/sd_engine.cpp): a full
    generation per call — both text encoders, steps guided denoising steps (the first
    eager, the rest hipGraph replays), the VAE decode — on random-init full-size weights;
    seconds_per_step = the mean device time of the replayed steps of the second call (the
    first autotunes the convolutions and captures the step)."""
    import numpy as np

    from ...sd_engine import NativeSD
    eng = NativeSD(".", version=version, dtype=dtype, device=device, random_init=True, seed=7)
    try:
        ids = np.full(77, 49407, dtype=np.int32)
        ids[0], ids[1:4] = 49406, (320, 1125, 539)
        unc = np.full(77, 49407, dtype=np.int32)
        unc[0] = 49406
        kw = dict(cond=ids, uncond=unc)
        if version in ("xl", "turbo"):
            kw.update(cond2=ids, uncond2=unc)
        n = steps + 1
        eng.generate(n_steps=n, guidance=7.5, seed=1, **kw)
        t0 = time.perf_counter()
        out = eng.generate(n_steps=n, guidance=7.5, seed=2, **kw)
        wall = time.perf_counter() - t0
    finally:
        eng.close()
    per = out.step_s[1:]
    return {"seconds_per_step": round(sum(per) / len(per), 5), "version": version,
            "resolution": f"{eng.width}x{eng.height}", "batch": 2, "dtype": dtype,
            "engine": "native", "steps": n, "per_step_s": [round(x, 5) for x in out.step_s],
            "text_ms": round(out.text_s * 1e3, 2), "vae_decode_ms": round(out.vae_s * 1e3, 2),
            "image_wall_s": round(wall, 4)}
