#!/bin/bash
# GPU box, round 5 (aa): LayerNorm folded into the SD transformer GEMMs (native engine):
# SD engine parity tests, then the native SDXL step with the fold on / off.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5aa; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { grep -E "^(FAILED|E  )|assert" $OUT/$name.log | head -40; [[ $name == sdt ]] || exit $rc; }; }
run kt 300 python -u -m pytest tests/test_sd_kernels_gpu.py -k "layernorm_folded" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/kt.log
run sdt 600 python -u -m pytest tests/test_sd_engine_gpu.py -q --maxfail=30 --timeout 300 --timeout-method thread
tail -2 $OUT/sdt.log
for f in 1 0 1 0; do
  CAKE_SD_LN_FOLD=$f run sd_$f 300 python -c "
from cake_amd.models.sd.bench import measure_native
import json; r = measure_native('xl', 8, 'f16', 0); print(json.dumps(r))"
  grep '^{' $OUT/sd_$f.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('fold $f', r.get('seconds_per_step'), min(r.get('per_step_s')))"
done
