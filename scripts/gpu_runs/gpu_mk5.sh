#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "0 0" "1 0"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin $1 --ring $2 --out gpurun_out/mk5_stamps_t$1_r$2.npy >> gpurun_out/mk5_stamps.log 2>&1 || exit $?
done
grep '^{' gpurun_out/mk5_stamps.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn_decode" > gpurun_out/mk5_attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mk5_attn_tests.log; exit $rc
