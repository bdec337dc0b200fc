"""Where does SDUnit.denoise spend wall time outside its steps? (host launch vs GPU)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.models.sd.config import get_config  # noqa: E402
from cake_amd.models.sd.schedulers import build_scheduler  # noqa: E402
from cake_amd.models.sd.shardable import SDUnit  # noqa: E402
from cake_amd.models.sd.weights import random_component  # noqa: E402

ver = sys.argv[1] if len(sys.argv) > 1 else "v1-5"
cfg = get_config(ver)
dev, dt = torch.device("cuda:0"), torch.float16
w = random_component("unet", cfg, dev, dt)
unit = SDUnit("unet", cfg, w, dev, dt)
sched = build_scheduler(cfg.scheduler, 12)
ts = sched.timesteps()
lat = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, device=dev)
ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim, device=dev, dtype=dt)
with torch.no_grad():
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, per = unit.denoise(lat, ctx, sched, ts, 7.5, True, rep)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {rep}: host {1e3 * (t1 - t0):.1f} ms, wall {1e3 * (t2 - t0):.1f} ms, "
              f"sum of steps {1e3 * sum(per):.1f} ms", flush=True)
    key = [k for k in unit._graphs if k[0] == "denoise"][0]
    g = unit._graphs[key]["graph"]
    torch.cuda.synchronize()
    for n in (1, 4):
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{n} replays: host {1e3 * (t1 - t0):.2f} ms, wall {1e3 * (t2 - t0):.2f} ms", flush=True)
