#!/bin/bash
# GPU box: decode-attention change A/B — previous library (cake_amd/lib/ab/libcake_kernels_old.so)
# vs the in-tree build: attention tests, phase stamps, decode at 32 / 176-context / 2048 prompts.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${AAB_OUT:-aab}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
OLD=$GRAFT_REPO_ROOT/cake_amd/lib/ab/libcake_kernels_old.so
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -5 $OUT/$name.log; exit $rc; }; }
run tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
tail -1 $OUT/tests.log
run stamps_new 240 env TKS=57,176,320,512,2048,4000 python scripts/attn_stamps.py
run stamps_old 240 env CAKE_KERNEL_LIB=$OLD TKS=57,176,320,512,2048,4000 python scripts/attn_stamps.py
for r in 1 2; do
  run d20_new_$r 200 python bench.py --no-extras --steps 20 --warmup 5
  run d20_old_$r 200 env CAKE_KERNEL_LIB=$OLD python bench.py --no-extras --steps 20 --warmup 5
  run d128_new_$r 200 python bench.py --no-extras
  run d128_old_$r 200 env CAKE_KERNEL_LIB=$OLD python bench.py --no-extras
done
run p2048_new 200 python bench.py --no-extras --prompt-len 2048
run p2048_old 200 env CAKE_KERNEL_LIB=$OLD python bench.py --no-extras --prompt-len 2048
exit 0
