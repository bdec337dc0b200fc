#!/bin/bash
# GPU box: register-staged decode attention — numerics, per-launch sweep, 8B decode at 32 / 2048.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn" > gpurun_out/r2s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2s_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A30 "Error\|FAILED" gpurun_out/r2s_pytest.log | head -80; exit $rc; fi
timeout -k 10 300 python scripts/bench_decode_attn.py > gpurun_out/attn_sweep.jsonl 2> gpurun_out/attn_sweep.err || { tail gpurun_out/attn_sweep.err; exit 1; }
cat gpurun_out/attn_sweep.jsonl
for P in 32 2048; do
  timeout -k 10 300 python bench.py --prompt-len $P --steps 64 --warmup 8 > gpurun_out/bench_p$P.json 2> gpurun_out/bench_p$P.err || { tail gpurun_out/bench_p$P.err; exit 1; }
  cat gpurun_out/bench_p$P.json
done
exit 0
