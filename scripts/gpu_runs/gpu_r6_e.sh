#!/bin/bash
# round 6: register-staged GEMM (cfg 21) numerics, then vs cfg 5 / table plan vs hipBLASLt
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6e; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run t21 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "22 or big_tile" --timeout 120 --timeout-method thread
run gemmrs 300 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 2048 --arms mfma,w4,w42,lib
cat $OUT/gemmrs.log
