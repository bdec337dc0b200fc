#!/bin/bash
# SD on the GPU box: kernel/model tests, then s/step for NCHW(MIOpen) vs NHWC(ours) eager vs graph.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_sd_gpu.py tests/test_sd_kernels_gpu.py -q -x > gpurun_out/t_sd.log 2>&1
r=$?; tail -4 gpurun_out/t_sd.log
if [[ $r -ne 0 ]]; then exit $r; fi
: > gpurun_out/sd_steps.jsonl
for v in ${VERSIONS:-v1-5 xl}; do
  CAKE_SD_NHWC=0 timeout -k 10 300 python scripts/bench_sd.py --version $v --steps 10 >> gpurun_out/sd_steps.jsonl 2>>gpurun_out/sd_steps.err || exit 1
  timeout -k 10 300 python scripts/bench_sd.py --version $v --steps 10 >> gpurun_out/sd_steps.jsonl 2>>gpurun_out/sd_steps.err || exit 1
  timeout -k 10 300 python scripts/bench_sd.py --version $v --steps 10 --graph --no-kv-cache >> gpurun_out/sd_steps.jsonl 2>>gpurun_out/sd_steps.err || exit 1
  timeout -k 10 300 python scripts/bench_sd.py --version $v --steps 10 --graph >> gpurun_out/sd_steps.jsonl 2>>gpurun_out/sd_steps.err || exit 1
done
cat gpurun_out/sd_steps.jsonl
