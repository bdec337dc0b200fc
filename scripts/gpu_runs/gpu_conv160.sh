#!/bin/bash
# GPU box: 160-output-channel halo conv tiles — tests, then the SDXL / SD1.5 steps (autotuned)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/conv160; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_sd_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv2d" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python - > $OUT/tuned.log 2>&1 <<'PY' || { tail $OUT/tuned.log; exit 1; }
import torch, collections
from cake_amd.models.sd.config import get_config
from cake_amd.models.sd.unet import UNet2DConditionModel
from cake_amd.models.sd.weights import random_component
from cake_amd.ops import conv as CV
cfg = get_config("xl"); dev = torch.device("cuda:0"); dt = torch.float16
w = random_component("unet", cfg, dev, dt); unet = UNet2DConditionModel(cfg.unet)
x = torch.randn(2, 4, 128, 128, device=dev, dtype=dt); ctx = torch.randn(2, 77, 2048, device=dev, dtype=dt)
with torch.no_grad():
    unet.forward(w, x, torch.full((), 999.0, device=dev), ctx, {})
torch.cuda.synchronize()
for k, v in CV.tuned().items():
    print(k[1:9], "->", v)
print(collections.Counter(v[0] for v in CV.tuned().values()))
PY
tail -3 $OUT/tuned.log
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/xl.log 2>&1 || { tail $OUT/xl.log; exit 1; }
grep '^{' $OUT/xl.log | tail -1 | cut -c1-150
timeout -k 10 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8 > $OUT/v15.log 2>&1 || { tail $OUT/v15.log; exit 1; }
grep '^{' $OUT/v15.log | tail -1 | cut -c1-150
