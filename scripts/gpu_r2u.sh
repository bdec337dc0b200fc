#!/bin/bash
# GPU box: Llama-3-70B decode on one GPU; 70B tensor-parallel rehearsal (2 ranks share the GPU).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --model llama3-70b --steps 32 --warmup 4 --max-seq 1024 > gpurun_out/bench70.json 2> gpurun_out/bench70.err || { tail gpurun_out/bench70.err; exit 1; }
cat gpurun_out/bench70.json
timeout -k 10 500 python bench.py --model llama3-70b --gpus 2 --dist-backend gloo --steps 32 --warmup 4 --max-seq 1024 > gpurun_out/bench70_tp2.json 2> gpurun_out/bench70_tp2.err || { tail gpurun_out/bench70_tp2.err; exit 1; }
cat gpurun_out/bench70_tp2.json
exit 0
