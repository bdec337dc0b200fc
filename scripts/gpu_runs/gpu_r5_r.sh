#!/bin/bash
# GPU box, round 5 (r): flash2 XCD-aware tile order (in-tree) and 3 workgroups/CU at head
# dim 64 (ab/ lb3) against the previous commit (ab/ old): tests, SD flash shapes, SDXL step.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5r; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run ft 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "flash" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/ft.log
CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_lb3.so run ft3 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "flash" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/ft3.log
for v in old new lb3; do
  case $v in old) export CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_old.so;; lb3) export CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_lb3.so;; *) unset CAKE_KERNEL_LIB;; esac
  run fl_$v 300 python scripts/bench_flash_split.py
  cat $OUT/fl_$v.log | python -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['ks0_us'], r['ks0_tflops'])"
  run sd_$v 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 6
  grep '^{' $OUT/sd_$v.log | cut -c1-120
done
