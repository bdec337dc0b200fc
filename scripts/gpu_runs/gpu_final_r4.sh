#!/bin/bash
# GPU box: end-of-round-4 records — the default bench line and the driver's flags, then
# rocprofv3 decode kernel tables (8B at 32 and 2048 prompt tokens) via gpu_prof_r3.sh.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/final4; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -15 $OUT/$name.log; exit $rc; }; }
run bench_default 400 python bench.py
grep '^{' $OUT/bench_default.log | cut -c1-300
run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep '^{' $OUT/bench_driver.log | cut -c1-300
bash scripts/gpu_prof_r3.sh || exit 1
