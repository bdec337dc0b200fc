#!/bin/bash
# Persistent decode ring engine: numerics, then phase stamps over loader settings, then step time.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mk_gpu.py > gpurun_out/mk4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mk4_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 0" "0 0"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin $1 --ring $2 --out gpurun_out/mk4_stamps_t$1_r$2.npy >> gpurun_out/mk4_stamps.log 2>&1 || exit $?
done
grep '^{' gpurun_out/mk4_stamps.log
timeout -k 10 240 python -u scripts/bench_mk.py --model llama3-8b --pos 32 1000 --reps 30 > gpurun_out/mk4_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/mk4_bench.log; exit $rc
