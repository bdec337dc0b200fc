#!/bin/bash
# round 5: our MFMA GEMM vs torch.matmul (hipBLASLt) on the Llama / SD shapes, no sweep
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python scripts/bench_gemm.py --inner 4 > gpurun_out/r5_gemm_vs_hipblaslt.jsonl 2> gpurun_out/r5_gemm_vs_hipblaslt.err || exit $?
cat gpurun_out/r5_gemm_vs_hipblaslt.jsonl
