#!/bin/bash
# GPU box, round 5 (i): 70B tp8 alone on one shared MI355X with the engine trace.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5i; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 CAKE_ENGINE_TRACE=1 CAKE_HOP_TIMEOUT=20
t0=$(date +%s)
timeout -k 10 300 python bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo --extras 70b_tp --no-sd --launch-timeout 280 > $OUT/n8.log 2> $OUT/n8.err
rc=$?
echo "== rc=$rc wall=$(( $(date +%s) - t0 ))s"
grep -v "control:\|decode " $OUT/n8.err | tail -60
grep '^{' $OUT/n8.log | cut -c1-600
exit $rc
