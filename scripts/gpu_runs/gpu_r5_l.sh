#!/bin/bash
# GPU box, round 5 (l): native SD engine parity tests (mini checkpoints).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5l; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_sd_engine_gpu.py -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "== tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $OUT/tests.log | head -60
exit $rc
