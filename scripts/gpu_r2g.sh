#!/bin/bash
# GPU box: full GPU test suite, 1-GPU bench, prefill TTFT, SDXL denoise-step kernel profile.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2g_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2g_pytest.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 300 python scripts/bench_prefill.py > gpurun_out/prefill.jsonl 2> gpurun_out/prefill.err || exit $?
cat gpurun_out/prefill.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sdxl" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_sd.py" --version xl --denoise --steps 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_sdxl.log" 2>&1 || exit $?
tail -2 "$GRAFT_REPO_ROOT/gpurun_out/prof_sdxl.log"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python scripts/bench_gemm.py --cfgs 0,8,11,9,5,1,10,6,12 > gpurun_out/gemm_il.jsonl 2> gpurun_out/gemm_il.err || exit $?
cat gpurun_out/gemm_il.jsonl
exit $rc
