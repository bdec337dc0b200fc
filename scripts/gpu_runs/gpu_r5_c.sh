#!/bin/bash
# GPU box, round 5 (c): 70B pp8 on the shared GPU with the engine's control-plane trace.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5c; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 CAKE_ENGINE_TRACE=1
t0=$(date +%s)
timeout -k 10 400 python bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo --extras 70b_pp --no-sd > $OUT/n8_70b.log 2>&1
echo "== n8_70b rc=$? wall=$(( $(date +%s) - t0 ))s"
grep '^{' $OUT/n8_70b.log | cut -c1-1500
grep "engine r" $OUT/n8_70b.log | tail -60
