#!/bin/bash
# GPU box, round 5 (y): flash2 at head dim 128 with one workgroup per CU (no VGPR spill)
# vs the previous two-per-CU bound (ab/ old): tests, causal prefill shapes, TTFT, SD shapes.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5y; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run ft 300 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_kernels_gpu.py -k "flash or prefill" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/ft.log
for v in old new; do
  if [[ $v == old ]]; then export CAKE_KERNEL_LIB=$PWD/ab/libcake_kernels_old.so; else unset CAKE_KERNEL_LIB; fi
  run fp_$v 300 python scripts/bench_flash_pairing.py
  cat $OUT/fp_$v.log | python -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        r=json.loads(l); print(r['H'], r['D'], r['N'], 'auto', r['auto_us'], r['auto_tflops'], 'unpaired', r['unpaired_us'], 'paired', r['paired_us'])"
  run fl_$v 300 python scripts/bench_flash_split.py
  grep sd15.l1 $OUT/fl_$v.log | cut -c1-140
  run pf_$v 300 python scripts/bench_prefill.py --lens 256,2048,4096 --reps 3
  grep prompt_len $OUT/pf_$v.log
done
