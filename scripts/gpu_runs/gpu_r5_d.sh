#!/bin/bash
# GPU box, round 5 (d): native engine GPU tests (TCP master, C-ABI worker, API over TCP
# workers, placement, teacher forcing) + the API-serving test.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5d; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_serving_gpu.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo "== tests rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
