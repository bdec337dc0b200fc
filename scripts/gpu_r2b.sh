#!/bin/bash
# GPU box: GEMM / sampling / pipeline tests, decode-attention microbench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_sampling_gpu.py tests/test_pipeline_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r2b.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/r2b.log | grep -v PASSED | head -20; tail -3 gpurun_out/r2b.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_decode_attn.py > gpurun_out/decode_attn.jsonl 2> gpurun_out/decode_attn.err || exit $?
cat gpurun_out/decode_attn.jsonl
exit $rc
