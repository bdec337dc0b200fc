#!/bin/bash
# GPU box, round 5 (q): flash2 loop fixes (next-tile loads after QK^T, K fragments read
# up front, permlane max, split row sums, f16 cvt_pk) — tests, then old (ab/) vs new lib on
# the SD flash shapes, the SDXL denoise step and Llama prefill.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5q; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run ft 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "flash" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/ft.log
for v in old new; do
  if [[ $v == old ]]; then export CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_old.so; else unset CAKE_KERNEL_LIB; fi
  run fl_$v 300 python scripts/bench_flash_split.py
  cat $OUT/fl_$v.log | python -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['ks0_us'], r['ks0_tflops'])"
  run sd_$v 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 6
  grep -i "ms" $OUT/sd_$v.log | tail -2
  run pf_$v 300 python scripts/bench_prefill.py --lens 256,2048 --reps 3
  cat $OUT/pf_$v.log | grep prompt_len
done
