#!/bin/bash
# round 5: native SD master with remote components, img2img through the worker's VAE
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_sd_engine_gpu.py -x -v --timeout 240 --timeout-method thread -k "remote_sd_components" > gpurun_out/r5_ai.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|assert" gpurun_out/r5_ai.log | tail -30; exit $rc
