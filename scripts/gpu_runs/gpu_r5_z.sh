#!/bin/bash
# GPU box, round 5 (z): GroupNorm NHWC stats slice size (CAKE_GN_SPLIT_PX) on the SDXL step
# (native engine, the bench's SD sub-record path) and the GN tests.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5z; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
for px in 16 64 128 32 16 64; do
  CAKE_GN_SPLIT_PX=$px run gt_$px 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "group_norm or groupnorm" -x -q --timeout 200 --timeout-method thread
  tail -1 $OUT/gt_$px.log
  CAKE_GN_SPLIT_PX=$px run sd_$px 300 python -c "
from cake_amd.models.sd.bench import measure_native
import json; r = measure_native('xl', 8, 'f16', 0); print(json.dumps(r))"
  grep '^{' $OUT/sd_$px.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('px $px', r.get('seconds_per_step'), min(r.get('per_step_s')))"
done
