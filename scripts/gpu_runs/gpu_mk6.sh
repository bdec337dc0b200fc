#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mk_gpu.py > gpurun_out/mk6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mk6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin 0 --out gpurun_out/mk6_stamps.npy > gpurun_out/mk6_stamps.log 2>&1 || exit $?
grep '^{' gpurun_out/mk6_stamps.log
timeout -k 10 240 python -u scripts/bench_mk.py --model llama3-8b --pos 32 1000 --reps 30 --thin 0 > gpurun_out/mk6_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/mk6_bench.log; exit $rc
