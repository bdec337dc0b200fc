#!/bin/bash
# GPU box, round 5 (u): LayerNorm gamma/beta prefetch — LN tests, SDXL step old (ab/) vs new.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5u; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run lt 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "layer_norm" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/lt.log
for v in old new old new; do
  if [[ $v == old ]]; then export CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_old.so; else unset CAKE_KERNEL_LIB; fi
  run sd_$v 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 6
  grep '^{' $OUT/sd_$v.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$v', r['value'], min(r['per_step_s']))"
done
