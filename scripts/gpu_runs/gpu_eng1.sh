#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_engine_gpu.py -k "pipeline or worker or tensor" > gpurun_out/eng1.log 2>&1 || { tail -60 gpurun_out/eng1.log; exit 1; }
tail -5 gpurun_out/eng1.log
