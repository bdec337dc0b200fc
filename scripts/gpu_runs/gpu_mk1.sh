#!/bin/bash
# First GPU check of the persistent decode: numerics tests, then the step microbench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mk_gpu.py > gpurun_out/mk1_tests.log 2>&1
rc=$?
tail -30 gpurun_out/mk1_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/bench_mk.py --model llama3-8b --pos 32 320 1000 2000 --reps 30 > gpurun_out/mk1_bench.log 2>&1
rc=$?
cat gpurun_out/mk1_bench.log | tail -20
exit $rc
