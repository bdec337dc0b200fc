#!/bin/bash
# round 5: library vs MFMA GEMM at short and off-grid prompt lengths (the plan table's
# nearest-M rule between the measured points)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python scripts/bench_gemm_lib.py --sweep-splits --ms 32,64,96,200,700,1500,2500 > gpurun_out/r5_gemm_lib_offgrid.jsonl 2> gpurun_out/r5_gemm_lib_offgrid.err || { tail -20 gpurun_out/r5_gemm_lib_offgrid.err; exit 1; }
cat gpurun_out/r5_gemm_lib_offgrid.jsonl
