#!/bin/bash
# GPU box, round 5 (x): native master failure detection (worker killed mid-session);
# vectorized prefill RoPE / KV write (tests + 8B prefill timing).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5x; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -40 $OUT/$name.log; exit $rc; }; }
run rt 300 python -u -m pytest tests/test_kernels_gpu.py -k "rope" -x -q --timeout 240 --timeout-method thread
tail -1 $OUT/rt.log
run fd 300 python -u -m pytest tests/test_engine_gpu.py -k "fails_loudly" -x -v --timeout 240 --timeout-method thread
grep -E "PASS|FAIL" $OUT/fd.log | tail -3
run pf 300 python scripts/bench_prefill.py --lens 256,2048 --reps 3
grep prompt_len $OUT/pf.log
