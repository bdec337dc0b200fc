#!/bin/bash
# GPU box: 8-phase GEMM tile correctness + per-cfg sweep vs the interleaved tiles.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r2n_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2n_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A25 "Error\|FAILED" gpurun_out/r2n_pytest.log | head -60; exit $rc; fi
timeout -k 10 300 python scripts/race_screen_gemm.py 14 30 > gpurun_out/race14.log 2>&1 || { cat gpurun_out/race14.log; exit 1; }
cat gpurun_out/race14.log
timeout -k 10 600 python scripts/bench_gemm.py --cfgs 0,5,14,6 > gpurun_out/gemm_8p.jsonl 2> gpurun_out/gemm_8p.err || exit $?
cat gpurun_out/gemm_8p.jsonl
exit 0
