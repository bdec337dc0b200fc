#!/bin/bash
# GPU-box check of the decode megakernel: numerics tests, then bench mega vs multi-kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_mega_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mega_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/mega_pytest.log
if [[ $rc -ne 0 ]]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
for m in 1 0; do
  CAKE_MEGA=$m timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_mega$m.json 2> gpurun_out/bench_mega$m.err
  b=$?; echo "CAKE_MEGA=$m"; cat gpurun_out/bench_mega$m.json; tail -2 gpurun_out/bench_mega$m.err
  if [[ $b -ne 0 ]]; then echo "bench rc=$b -> stop"; exit $b; fi
done
