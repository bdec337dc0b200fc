#!/bin/bash
# GPU box, round 5 (b): the attention error-word test, then shared-GPU rehearsals of the
# default multi-rank bench on the native engine (N ranks on the one GPU: gloo for the
# bench's own barrier / max; the engines' hops and all-reduces are device-side IPC).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5b; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; local t0=$(date +%s); timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc wall=$(( $(date +%s) - t0 ))s"; [[ $rc -eq 0 ]] || { tail -25 $OUT/$name.log; exit $rc; }; }
run attn_err 300 python -u -m pytest tests/test_engine_gpu.py -k "attention_error_word or continue_equals" -v --timeout 200 --timeout-method thread
run n2 600 python bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo
grep '^{' $OUT/n2.log | cut -c1-2500
run n8 900 python bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo
grep '^{' $OUT/n8.log | cut -c1-3000
