#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sd_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/r5_aq.log 2>&1
rc=$?; tail -3 gpurun_out/r5_aq.log; exit $rc
