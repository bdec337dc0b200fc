#!/bin/bash
# GPU box: SD denoise steps + prefill TTFT with the measured GEMM plans; SDXL step profile.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/sd_bench.jsonl
for v in v1-5 xl; do
  timeout -k 10 300 python scripts/bench_sd.py --version $v --denoise --steps 10 >> gpurun_out/sd_bench.jsonl 2>> gpurun_out/sd_bench.err || exit $?
done
cat gpurun_out/sd_bench.jsonl
timeout -k 10 300 python scripts/bench_prefill.py > gpurun_out/prefill.jsonl 2> gpurun_out/prefill.err || exit $?
cat gpurun_out/prefill.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sdxl2" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_sd.py" --version xl --denoise --steps 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_sdxl2.log" 2>&1 || exit $?
exit 0
