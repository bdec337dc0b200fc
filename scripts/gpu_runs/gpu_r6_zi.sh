#!/bin/bash
# round 6: GEMM workspace sized by the kernel library's split plan: GEMM / engine / SD tests, TTFT
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zi; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_sd_engine_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for P in 512 2048; do
  timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print($P, r['ttft_ms_prefill'], r['value'], r['hbm_used_mib'])"
done
