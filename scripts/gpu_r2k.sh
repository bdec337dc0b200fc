#!/bin/bash
# GPU box: GEMM tests (incl. the 4-wave 256x256 interleaved tile), per-cfg sweep, denoise wall diagnosis.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r2k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2k_pytest.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 600 python scripts/bench_gemm.py --cfgs 0,5,14,6,1,4,12,13 > gpurun_out/gemm_c14.jsonl 2> gpurun_out/gemm_c14.err || exit $?
cat gpurun_out/gemm_c14.jsonl
timeout -k 10 300 python scripts/diag_denoise.py v1-5 > gpurun_out/diag_denoise.log 2>&1 || exit $?
cat gpurun_out/diag_denoise.log
exit 0
