#!/bin/bash
# round end: the whole GPU suite + smoke (scripts/gpu_full.sh), then the default bench
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
bash scripts/gpu_full.sh 1000 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -30 gpurun_out/final/bench.err; exit 1; }
tail -1 gpurun_out/final/bench.json
