#!/bin/bash
# round 6: deep-staged four-wave GEMM (cfg 25-27): numerics, then A/B against the
# single-region four-wave tiles (22-24), the table's MFMA plan and the library GEMM
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6j; mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "25 or 26 or 27"
run arms 500 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 2048 --arms mfma,w4,d4,w3,d3,w1,d1,w42,d42,lib
cat $OUT/arms.log
