#!/bin/bash
# GPU box: kernel tests (GEMM, attention, sampling), GEMM sweep, decode-attention microbench, bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_sampling_gpu.py tests/test_model_gpu.py tests/test_parity_hf.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c.log 2>&1
rc=$?; tail -5 gpurun_out/r2c.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_decode_attn.py > gpurun_out/decode_attn.jsonl 2> gpurun_out/decode_attn.err || exit $?
cat gpurun_out/decode_attn.jsonl
timeout -k 10 600 python scripts/bench_gemm.py --sweep > gpurun_out/gemm_sweep.jsonl 2> gpurun_out/gemm_sweep.err || exit $?
cat gpurun_out/gemm_sweep.jsonl
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --prompt-len 2048 --steps 64 --warmup 8 > gpurun_out/bench2048.json 2> gpurun_out/bench2048.err || exit $?
cat gpurun_out/bench2048.json
exit $rc
