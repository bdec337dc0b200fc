#!/bin/bash
# round 6 final: the whole GPU suite as the driver runs it
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6final5; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 ${1:-1150} python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -5 $OUT/pytest.log; exit $rc
