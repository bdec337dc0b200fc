#!/bin/bash
# decode steps per graph replay A/B (8B, default flags otherwise)
set -o pipefail
mkdir -p gpurun_out/k
export PYTHONUNBUFFERED=1
for k in 1 4 8 1 4 8; do
  timeout -k 10 300 python -u bench.py --no-extras --no-sd --steps 128 --warmup 16 --steps-per-graph $k \
    > gpurun_out/k/bench_$k.log 2>&1 || { tail -20 gpurun_out/k/bench_$k.log; exit 1; }
  echo "k=$k $(grep '^{' gpurun_out/k/bench_$k.log | tail -1 | cut -c1-160)"
done
