#!/bin/bash
# GPU box: GEMM tests + per-shape config sweep vs hipBLASLt.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 600 python scripts/bench_gemm.py --sweep > gpurun_out/gemm_sweep.jsonl 2> gpurun_out/gemm_sweep.err || exit $?
cat gpurun_out/gemm_sweep.jsonl
