#!/bin/bash
# round 6: smoke on the native engine, the pipeline / TP / engine tests (prefill relay
# buffers and their self-test, the forced-failure fallback), SD v2-1 on the native engine
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6a; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run pipe 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread
run sd21 400 python -u -m pytest tests/test_sd_engine_gpu.py -x -v -k "v2-1" --timeout 300 --timeout-method thread
