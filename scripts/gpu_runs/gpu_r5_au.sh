#!/bin/bash
# round 5: library vs MFMA GEMM on the tensor-parallel ranks' prefill slices (tp 2 / 4 / 8)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python scripts/bench_gemm_lib.py --tp 2,4,8 --sweep-splits --ms 128,512,1024,2048,4096 > gpurun_out/r5_gemm_lib_tp.jsonl 2> gpurun_out/r5_gemm_lib_tp.err || { tail -20 gpurun_out/r5_gemm_lib_tp.err; exit 1; }
wc -l gpurun_out/r5_gemm_lib_tp.jsonl
