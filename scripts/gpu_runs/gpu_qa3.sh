#!/bin/bash
# VAE kernels + decoder buckets (tests), then the fused-QKV+attention kernel table A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_sd_kernels_gpu.py -k "conv1x1 or small_ic or out_nchw" \
  > gpurun_out/qa3_sdk.log 2>&1 || { tail -30 gpurun_out/qa3_sdk.log; exit 1; }
tail -1 gpurun_out/qa3_sdk.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_sd_gpu.py tests/test_model_gpu.py > gpurun_out/qa3_model.log 2>&1 || { tail -40 gpurun_out/qa3_model.log; exit 1; }
tail -1 gpurun_out/qa3_model.log
bash scripts/gpu_qa2.sh
