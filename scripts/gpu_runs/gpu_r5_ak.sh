#!/bin/bash
# round 5: library GEMM tests (incl. the torch-free process)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -k "library" > gpurun_out/r5_ak.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/r5_ak.log | tail -12; exit $rc
