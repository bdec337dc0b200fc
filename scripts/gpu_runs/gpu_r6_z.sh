#!/bin/bash
# round 6: wide epilogue read-out in gemm_kernel (64 / 128-column wave tiles): numerics
# (GEMM + the SD and engine tests that run the GEMMs), A/B on the SD step and prefill
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6z; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_sd_engine_gpu.py tests/test_engine_gpu.py -k "not dead and not tcp" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
SD='import json; from cake_amd.models.sd.bench import measure_native as m; r = m("xl", 8); print(json.dumps({k: r[k] for k in ("seconds_per_step", "per_step_s")}))'
timeout -k 10 300 python -c "$SD" > $OUT/sdxl.log 2>&1 || { tail -20 $OUT/sdxl.log; exit 1; }
tail -1 $OUT/sdxl.log
for P in 512 2048; do
  timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print($P, r['ttft_ms_prefill'], r['value'])"
done
