#!/bin/bash
# GPU box: decode tok/s with 1 vs 4 decode steps per graph replay (interleaved)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/kab; mkdir -p $OUT
i=0
for k in 1 4 1 4; do
  i=$((i + 1))
  timeout -k 10 200 python bench.py --no-extras --steps 128 --warmup 16 --steps-per-graph $k > $OUT/r$i.log 2>&1 || { tail -5 $OUT/r$i.log; exit 1; }
  echo "k=$k $(grep '^{' $OUT/r$i.log | cut -c1-110)"
done
