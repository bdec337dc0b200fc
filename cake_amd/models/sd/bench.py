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


_SPLIT_SEQ = [0]


def measure_native_split(env, version: str = "xl", steps: int = 8, dtype: str = "f16",
                         owners=None) -> dict | None:
    """BASELINE config 5 on the native engine: the UNet's stages split over env.world ranks
    (one process per GPU, sd_engine.h CakeSdSplitOpts), each denoise step one graph replay
    per rank with device bulk hops; rank 0 runs the text encoders, the scheduler and the
    VAE.  Seconds per diffusion step = rank 0's device time of the replayed steps of the
    second generation (its step graph waits for the prediction of the last rank).  Rank 0
    gets the record, the others None."""
    import os

    import numpy as np

    from ...sd_engine import NativeSD
    _SPLIT_SEQ[0] += 1
    port = int(os.environ.get("MASTER_PORT", "29500")) + 300 + _SPLIT_SEQ[0]
    addr = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{port}"
    dev = (env.dev.index or 0) if getattr(env, "dev", None) is not None else 0
    t0 = time.perf_counter()
    eng = NativeSD(".", version=version, dtype=dtype, device=dev, random_init=True, seed=7,
                   rank=env.rank, world=env.world, master_addr=addr, owners=owners,
                   connect_timeout_s=180.0)
    out = None
    try:
        info = eng.split_info()
        if env.rank == 0:
            ids = np.full(77, 49407, dtype=np.int32)
            ids[0], ids[1:4] = 49406, (320, 1125, 539)
            unc = np.full(77, 49407, dtype=np.int32)
            unc[0] = 49406
            kw = dict(cond=ids, uncond=unc)
            if version in ("xl", "turbo"):
                kw.update(cond2=ids, uncond2=unc)
            n = steps + 1
            eng.generate(n_steps=n, guidance=7.5, seed=1, **kw)
            t1 = time.perf_counter()
            img = eng.generate(n_steps=n, guidance=7.5, seed=2, **kw)
            wall = time.perf_counter() - t1
            per = img.step_s[1:]
            n_st = info["stages"]
            runs = {}
            for k in range(n_st):
                r = int(k * info["ranks_used"] / n_st) if owners is None else int(owners[k])
                runs.setdefault(str(r), []).append(k)
            out = {"seconds_per_step": round(sum(per) / len(per), 5), "engine": "native",
                   "transport": "ipc-bulk", "version": version, "batch": 2, "dtype": dtype,
                   "resolution": f"{eng.width}x{eng.height}", "steps": n,
                   "ranks_used": info["ranks_used"], "stage_runs": runs,
                   "per_step_s": [round(x, 5) for x in img.step_s],
                   "image_wall_s": round(wall, 4),
                   "setup_s": round(t1 - t0, 2),
                   "latent_checksum": float(np.asarray(img.latents, dtype=np.float64).sum())}
            eng.close()  # the workers leave serve()
        else:
            eng.serve()
            eng.close()
    finally:
        eng.close()
    return out
