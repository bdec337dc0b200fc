#!/bin/bash
# GPU box: SD + attention + pipeline tests, decode-attention microbench, SD step bench, decode bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_sd_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2d.log 2>&1
rc=$?; tail -5 gpurun_out/r2d.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_decode_attn.py > gpurun_out/decode_attn.jsonl 2> gpurun_out/decode_attn.err || exit $?
cat gpurun_out/decode_attn.jsonl
timeout -k 10 400 python scripts/bench_sd.py > gpurun_out/sd_bench.jsonl 2> gpurun_out/sd_bench.err || exit $?
cat gpurun_out/sd_bench.jsonl
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
exit $rc
