#!/bin/bash
# native engine + 12-wave attention + fused QKV/attention + VAE kernels: tests, then kernel tables
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_engine_gpu.py > gpurun_out/qa5_engine.log 2>&1 || { tail -40 gpurun_out/qa5_engine.log; exit 1; }
tail -3 gpurun_out/qa5_engine.log
bash scripts/gpu_qa4.sh
