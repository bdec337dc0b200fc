#!/bin/bash
# GPU box: pipeline (multi-rank on one GPU) + GEMM tests, GEMM bench, decode kernel profiles.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pipe.log 2>&1
rc=$?; tail -15 gpurun_out/pipe.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err || exit $?
cat gpurun_out/gemm_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof32" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 4 > "$GRAFT_REPO_ROOT/gpurun_out/prof32.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof2048" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 4 --prompt-len 2048 > "$GRAFT_REPO_ROOT/gpurun_out/prof2048.log" 2>&1 || exit $?
exit $rc
