#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_sd_engine_gpu.py -x -v --timeout 240 --timeout-method thread -k "remote or dies" > gpurun_out/r5_aw.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/r5_aw.log | tail -12; exit $rc
