#!/bin/bash
# GPU box, round 5 (s): native SD engine tests (incl. bsize 2 + intermediary images).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5s; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -40 $OUT/$name.log; exit $rc; }; }
run sdt 600 python -u -m pytest tests/test_sd_engine_gpu.py -x -v --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|ERROR" $OUT/sdt.log | tail -30
