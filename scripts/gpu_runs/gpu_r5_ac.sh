#!/bin/bash
# GPU box, round 5 (ac): head-parallel decode attention at a 2048-token context (8B decode
# bench, --prompt-len 2048): the split-K path vs CAKE_ATTN_HEADS=4096:{4,8,16}.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ac; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run kt 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode_heads" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/kt.log
for h in 0 4096:16:4 4096:8:4 4096:4:4 4096:16 0; do
  tag=${h//:/_}
  CAKE_ATTN_HEADS=$h run b_$tag 300 python bench.py --no-extras --no-sd --prompt-len 2048 --steps 64 --warmup 8
  grep '^{' $OUT/b_$tag.log | cut -c1-130
done
