#!/bin/bash
# GPU box, round 5 (h): the full default N=8 bench on ONE shared MI355X (gloo control
# plane; device hops / all-reduces over IPC), every sub-record: 8B pp / tp / pp_streams,
# 70B pp / tp, SDXL split over 8 ranks.  Wall time against the driver's 600 s.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5h; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 CAKE_ENGINE_TRACE=1
( while sleep 50; do echo "$(date +%T) alive" >> $OUT/heartbeat.txt; done ) &
HB=$!
t0=$(date +%s)
timeout -k 10 1080 python bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo --launch-timeout 1050 > $OUT/n8.log 2> $OUT/n8.err
rc=$?
t1=$(date +%s)
kill $HB
echo "== n8 rc=$rc wall=$((t1 - t0))s"
grep '^{' $OUT/n8.log > $OUT/n8.json || tail -40 $OUT/n8.err
exit $rc
