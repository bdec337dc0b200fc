#!/bin/bash
# round 5: causal flash attention with a forced key split vs the paired default
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/bench_flash_causal_split.py > gpurun_out/r5_flash_causal_split.jsonl 2> gpurun_out/r5_flash_causal_split.err || { tail -20 gpurun_out/r5_flash_causal_split.err; exit 1; }
cat gpurun_out/r5_flash_causal_split.jsonl
