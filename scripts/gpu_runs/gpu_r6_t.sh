#!/bin/bash
# round 6: k-loop segment stamps of the four-wave 256x256 GEMM (diagnostic build)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6t; mkdir -p $OUT
for s in "8192 8192 8192" "4096 4096 4096" "2048 8192 28672"; do
  timeout -k 10 60 ./scripts/gemm_stamp $s | tee -a $OUT/stamps.jsonl || exit 1
done
