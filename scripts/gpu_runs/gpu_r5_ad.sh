#!/bin/bash
# GPU box, round 5 (ad): 8B decode kernel tables at a 2048-token context, split-K attention
# vs the head-parallel launch (16 waves, prefetch 4).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ad; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for h in 0 4096:16:4; do
  tag=${h//:/_}
  CAKE_ATTN_HEADS=$h timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/p_$tag" -o run -- python3 "$ROOT/bench.py" --no-extras --no-sd --prompt-len 2048 --steps 64 --warmup 4 > "$ROOT/$OUT/p_$tag.log" 2>&1 || { tail -20 "$ROOT/$OUT/p_$tag.log"; exit 1; }
  DB=$(find "$ROOT/$OUT/p_$tag" -name '*.db' | head -n 1)
  python3 "$ROOT/scripts/decode_kernel_table.py" "$DB" --ctx 2084 > "$ROOT/$OUT/t_$tag.txt"
  echo "=== $h"; cat "$ROOT/$OUT/t_$tag.txt"
  find "$ROOT/$OUT/p_$tag" -name '*.db' -delete
done
