#!/bin/bash
# GPU box, round 5 (k): SDXL denoise step kernel breakdown (rocprofv3 --kernel-trace --stats).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5k; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 1; }
tail -3 $OUT/plain.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/bench_sd.py" --version xl --denoise --graph --steps 8 > "$ROOT/$OUT/prof.log" 2>&1 || { tail -20 "$ROOT/$OUT/prof.log"; exit 1; }
db=$(find "$ROOT/$OUT/prof" -name '*.db' | head -n 1)
python3 "$ROOT/scripts/kernel_stats_db.py" "$db" --top 32 --per 8 --last-ms 240 > "$ROOT/$OUT/sdxl_step_kernels.txt" && cat "$ROOT/$OUT/sdxl_step_kernels.txt"
find "$ROOT/$OUT/prof" -name '*.db' -delete
