#!/bin/bash
# decode attention split target A/B at long context (prefetch auto)
set -o pipefail
mkdir -p gpurun_out/tgt
export PYTHONUNBUFFERED=1
for pl in 4000 1024; do
  for t in 16 24 32 16 24 32; do
    CAKE_ATTN_TARGET=$t timeout -k 10 300 python -u bench.py --no-extras --no-sd --steps 96 --warmup 16 --prompt-len $pl \
      > gpurun_out/tgt/bench_${pl}_$t.log 2>&1 || { tail -20 gpurun_out/tgt/bench_${pl}_$t.log; exit 1; }
    echo "prompt=$pl target=$t $(grep '^{' gpurun_out/tgt/bench_${pl}_$t.log | tail -1 | cut -c1-110)"
  done
done
