#!/bin/bash
# round 5: rope / rmsnorm / prefill attention tests, then the 8B prefill kernel table at 2048
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ao; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rope or rmsnorm" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [[ $rc -eq 0 ]] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/bench_prefill.py" --lens 2048 --reps 3 > "$ROOT/$OUT/prof.log" 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
DB=$(find "$OUT/prof" -name '*.db' | head -n 1)
python3 scripts/kernel_stats_db.py "$DB" --last-ms 29 --top 25 > $OUT/prefill2048.txt
cat $OUT/prefill2048.txt
find $OUT -name '*.db' -delete
