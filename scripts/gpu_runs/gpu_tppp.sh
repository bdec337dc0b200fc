#!/bin/bash
# tightened multi-rank equivalence (teacher-forced logits, >= 32 steps): TP and PP on
# the shared GPU
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_tp_gpu.py tests/test_pipeline_gpu.py > gpurun_out/tppp.log 2>&1 || { tail -60 gpurun_out/tppp.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/tppp.log | tail -30
