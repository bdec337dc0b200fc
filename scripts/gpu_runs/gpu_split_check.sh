#!/bin/bash
# GPU box: after splitting gemv / gemm into several translation units — decode / GEMM / engine
# tests, smoke, the driver-flag bench line
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/splitck; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engine_gpu.py tests/test_gemm_gpu.py tests/test_sampling_gpu.py -x -q --timeout 120 --timeout-method thread
tail -1 $OUT/tests.log
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras
grep '^{' $OUT/bench.log | cut -c1-200
