#!/bin/bash
# round 6: SDXL step GEMM plans re-tuned on the final kernels (four-wave remainder pair in the
# candidates); SDXL step before / after
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zm; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
SD='import json; from cake_amd.models.sd.bench import measure_native as m; r = m("xl", 8); print(json.dumps({k: r[k] for k in ("seconds_per_step",)}))'
run before 300 python -c "$SD"
run tune 900 python scripts/tune_sd_gemm.py --versions xl,v1-5 --write $OUT/gemm_tuned.json
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
run after 300 python -c "$SD"
grep step_gemm $OUT/tune.log
