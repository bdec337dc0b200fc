#!/bin/bash
# round end: 8B decode kernel table at a short (32-token) prompt, the default bench path
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5at; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/p" -o run -- python3 "$ROOT/bench.py" --no-extras --no-sd --prompt-len 32 --steps 64 --warmup 4 > "$ROOT/$OUT/p.log" 2>&1 || { tail -20 "$ROOT/$OUT/p.log"; exit 1; }
DB=$(find "$ROOT/$OUT/p" -name '*.db' | head -n 1)
python3 "$ROOT/scripts/decode_kernel_table.py" "$DB" --ctx 68 > "$ROOT/$OUT/t.txt"
cat "$ROOT/$OUT/t.txt"
find "$ROOT/$OUT/p" -name '*.db' -delete
