#!/bin/bash
# GPU box: GEMM correctness (all epilogues / cfgs) then the per-cfg sweep (AGPR-pinned accumulators vs not).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemm_ag_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_ag_tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 700 python scripts/bench_gemm.py --cfgs 0,10,5,11,8,9,6,2,1,4 > gpurun_out/gemm_ag.jsonl 2> gpurun_out/gemm_ag.err || exit $?
cat gpurun_out/gemm_ag.jsonl
