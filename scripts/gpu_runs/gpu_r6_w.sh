#!/bin/bash
# round 6: four-wave epilogue stamps with / without the store drain
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6w; mkdir -p $OUT
for s in "8192 8192 8192" "4096 4096 4096"; do
  timeout -k 10 60 ./scripts/gemm_stamp $s | tee -a $OUT/stamps.jsonl || exit 1
  timeout -k 10 60 ./scripts/gemm_stamp_nodrain $s | tee -a $OUT/stamps_nodrain.jsonl || exit 1
done
