#!/bin/bash
# round 6: native img2img at bsize 1 / 2 against the Python pipeline
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6k; mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run img2img 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_sd_engine_gpu.py -k "img2img"
