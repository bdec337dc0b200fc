#!/bin/bash
# round 6 last check: SD tests on the re-tuned SD plans, smoke, default bench
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zo; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sd_engine_gpu.py tests/test_sd_gpu.py tests/test_sd_split_native_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
