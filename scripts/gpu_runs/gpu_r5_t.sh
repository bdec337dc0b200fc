#!/bin/bash
# GPU box, round 5 (t): the default bench line as the driver runs it at N=1.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5t; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
(while sleep 50; do date >> $OUT/heartbeat; done) & HB=$!
start=$(date +%s)
timeout -k 10 900 python bench.py > $OUT/bench.log 2>&1
rc=$?
kill $HB 2>/dev/null
echo "rc=$rc wall_s=$(( $(date +%s) - start ))"
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json || true
cut -c1-3000 $OUT/bench.json
[[ $rc -eq 0 ]] || tail -30 $OUT/bench.log
exit $rc
