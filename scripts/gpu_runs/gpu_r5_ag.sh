#!/bin/bash
# round 5: library GEMM path (hipBLASLt) tests, then ours vs library across prefill lengths
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k library --timeout 120 --timeout-method thread > gpurun_out/r5_lib_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_lib_tests.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 600 python scripts/bench_gemm_lib.py > gpurun_out/r5_gemm_lib.jsonl 2> gpurun_out/r5_gemm_lib.err || { tail -20 gpurun_out/r5_gemm_lib.err; exit 1; }
cat gpurun_out/r5_gemm_lib.jsonl
