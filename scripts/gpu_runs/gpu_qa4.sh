#!/bin/bash
# 12-wave attention core 2 + fused QKV/attention + VAE kernels: tests, then kernel tables
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_sd_kernels_gpu.py tests/test_sampling_gpu.py -k "attn or qkv or conv1x1 or small_ic or out_nchw or full_mass" \
  > gpurun_out/qa4_k.log 2>&1 || { tail -30 gpurun_out/qa4_k.log; exit 1; }
tail -1 gpurun_out/qa4_k.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_sd_gpu.py tests/test_model_gpu.py tests/test_mk_gpu.py > gpurun_out/qa4_model.log 2>&1 || { tail -40 gpurun_out/qa4_model.log; exit 1; }
tail -1 gpurun_out/qa4_model.log
bash scripts/gpu_qa2.sh
