#!/bin/bash
# fused QKV + attention: numerics, decoder buckets, then the 8B decode bench A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "qkv_attn or qkv_rope or attn_decode_merge" tests/test_model_gpu.py \
  > gpurun_out/qa1_tests.log 2>&1 || { tail -30 gpurun_out/qa1_tests.log; exit 1; }
tail -3 gpurun_out/qa1_tests.log
for on in 0 1 0 1; do
  CAKE_QKV_ATTN=$on timeout -k 10 300 python -u bench.py --no-extras --no-sd --steps 128 --warmup 16 \
    > gpurun_out/qa1_bench_$on.log 2>&1 || { tail -20 gpurun_out/qa1_bench_$on.log; exit 1; }
  echo "qkv_attn=$on $(grep '^{' gpurun_out/qa1_bench_$on.log | tail -1 | cut -c1-200)"
done
