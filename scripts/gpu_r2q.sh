#!/bin/bash
# GPU box: split x prologue + weight prefetch for the decode GEMVs — numerics, then in-graph decode tok/s sweep.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemv or swiglu or qkv or norm" > gpurun_out/r2q_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2q_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A30 "Error\|FAILED" gpurun_out/r2q_pytest.log | head -80; exit $rc; fi
timeout -k 10 600 python scripts/sweep_decode_tuning.py > gpurun_out/pf_sweep.jsonl 2> gpurun_out/pf_sweep.err || { tail -20 gpurun_out/pf_sweep.err; exit 1; }
cat gpurun_out/pf_sweep.jsonl
exit 0
