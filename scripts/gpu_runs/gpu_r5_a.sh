#!/bin/bash
# GPU box, round 5 (a): the native-engine bench (driver flags; python-engine A/B), then the
# native engine GPU tests (placement, teacher-forced TP / bf16 hops, error word, continue)
# and the API-serving test.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5a; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -25 $OUT/$name.log; exit $rc; }; }
run bench_native 400 python bench.py --gpus 1 --steps 20 --warmup 5
grep '^{' $OUT/bench_native.log | cut -c1-900
run bench_python 300 python bench.py --gpus 1 --steps 20 --warmup 5 --engine python --no-sd --no-extras
grep '^{' $OUT/bench_python.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_serving_gpu.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo "== tests rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
