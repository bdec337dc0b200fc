#!/bin/bash
# round 6: ping-pong GEMM (cfg 20) vs cfg 5 / table plan vs hipBLASLt, plus its GPU tests
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6b; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run gemmpp 300 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 2048
cat $OUT/gemmpp.log
