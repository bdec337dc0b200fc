#!/bin/bash
# GPU box: SD + sampling + model tests, SD denoise bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_sd_gpu.py tests/test_sampling_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f.log 2>&1
rc=$?; tail -5 gpurun_out/r2f.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
for v in v1-5 xl; do
  timeout -k 10 300 python scripts/bench_sd.py --version $v --denoise >> gpurun_out/sd_bench.jsonl 2>> gpurun_out/sd_bench.err || exit $?
done
cat gpurun_out/sd_bench.jsonl
exit $rc
