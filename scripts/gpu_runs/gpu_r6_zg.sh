#!/bin/bash
# round 6: four-wave remainder-pair numerics + the engine tests that run the new plans
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zg; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_engine_gpu.py -k "pair or remainder or prefill or matches" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; exit $rc
