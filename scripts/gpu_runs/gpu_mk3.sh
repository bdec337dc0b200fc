#!/bin/bash
# Persistent decode ring engine: phase stamps and step time over loader settings.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "1 0" "0 0" "1 4"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin $1 --ring $2 --out gpurun_out/mk3_stamps_t$1_r$2.npy >> gpurun_out/mk3_stamps.log 2>&1 || exit $?
done
grep '^{' gpurun_out/mk3_stamps.log
