#!/bin/bash
# GPU box: 8B decode tok/s vs live context (prompt lengths 32 .. 8000, max_seq 8192) and
# 70B at a 2048-token prompt: one JSON line per point into gpurun_out/ctx/.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ctx; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for P in 32 256 512 1024 2048 4096 8000; do
  timeout -k 10 200 python bench.py --no-extras --steps 64 --warmup 8 --prompt-len $P --max-seq 8192 > $OUT/p$P.log 2>&1 || { tail -3 $OUT/p$P.log; exit 1; }
  grep -h '^{' $OUT/p$P.log | cut -c1-140
done
timeout -k 10 300 python bench.py --no-extras --model llama3-70b --steps 32 --warmup 4 --prompt-len 2048 > $OUT/p70b_2048.log 2>&1 || { tail -3 $OUT/p70b_2048.log; exit 1; }
grep -h '^{' $OUT/p70b_2048.log | cut -c1-140
exit 0
