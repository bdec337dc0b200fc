#!/bin/bash
# GPU box, round 5 (w): kernel table of 8B prefill at 2048 tokens (bench_prefill, 3 reps:
# the last 30 ms window = one prefill).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5w; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/bench_prefill.py" --lens 2048 --reps 3 > "$ROOT/$OUT/prof.log" 2>&1 || { tail -20 "$ROOT/$OUT/prof.log"; exit 1; }
DB=$(find "$ROOT/$OUT/prof" -name '*.db' | head -n 1)
python3 "$ROOT/scripts/kernel_stats_db.py" "$DB" --last-ms 31 --top 25 > "$ROOT/$OUT/prefill2048.txt"
cat "$ROOT/$OUT/prefill2048.txt"
find "$ROOT/$OUT" -name '*.db' -delete
