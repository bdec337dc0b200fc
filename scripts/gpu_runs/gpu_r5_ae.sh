#!/bin/bash
# GPU box, round 5 (ae): native SD master over a TCP worker serving the UNet and the VAE,
# then the whole SD engine test file.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ae; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -40 $OUT/$name.log; exit $rc; }; }
run rm 400 python -u -m pytest tests/test_sd_engine_gpu.py -k "remote_sd_components" -x -v --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|SKIP" $OUT/rm.log | tail -4
run sdt 600 python -u -m pytest tests/test_sd_engine_gpu.py -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/sdt.log
