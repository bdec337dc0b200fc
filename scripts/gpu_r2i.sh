#!/bin/bash
# GPU box: GEMM + TP tests (incl. the nccl path under torchrun), full (cfg, split-K) GEMM sweep.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_tp_gpu.py -x -v --timeout 170 --timeout-method thread > gpurun_out/r2i_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2i_pytest.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 900 python scripts/bench_gemm.py --sweep > gpurun_out/gemm_sweep_full.jsonl 2> gpurun_out/gemm_sweep_full.err || exit $?
cat gpurun_out/gemm_sweep_full.jsonl
exit 0
