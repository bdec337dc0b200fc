#!/bin/bash
# Persistent decode: numerics, step microbench, phase stamps.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mk_gpu.py > gpurun_out/mk_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/bench_mk.py --model llama3-8b --pos 32 1000 --reps 30 > gpurun_out/mk_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/mk_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --out gpurun_out/mk_stamps_p32.npy > gpurun_out/mk_stamps.log 2>&1
rc=$?; grep '^{' gpurun_out/mk_stamps.log; exit $rc
