#!/bin/bash
# round 5: captured text encoders in the native SD engine: SD engine tests, then the SD
# record of the bench (text_ms, image wall) twice (the first generation captures)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ar; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_sd_engine_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --extras sd > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
python -c "
import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(json.dumps(r.get('sd')))"
