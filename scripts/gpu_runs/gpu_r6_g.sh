#!/bin/bash
# round 6: four-wave tiles (256x256 cfg 22, 256x192 cfg 23) with and without the in-kernel
# split-K pair vs the tuned plan and hipBLASLt on the 8B / 70B prefill shapes at 2048 tokens
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6g; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run t23 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "23 or pair" --timeout 120 --timeout-method thread
run arms 400 python scripts/bench_gemm_pp.py --shapes 8b,70b --ms 2048 --arms mfma,w4,w42,w3,w32,lib
cat $OUT/arms.log
