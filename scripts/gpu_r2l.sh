#!/bin/bash
# GPU box: full GPU suite, 1-GPU bench, decode GEMV in-graph tuning sweep, SD denoise bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 170 --timeout-method thread > gpurun_out/r2l_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2l_pytest.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 600 python scripts/sweep_decode_tuning.py > gpurun_out/decode_tuning.jsonl 2> gpurun_out/decode_tuning.err || exit $?
cat gpurun_out/decode_tuning.jsonl
rm -f gpurun_out/sd_bench.jsonl
for v in v1-5 xl; do
  timeout -k 10 300 python scripts/bench_sd.py --version $v --denoise --steps 10 >> gpurun_out/sd_bench.jsonl 2>> gpurun_out/sd_bench.err || exit $?
done
cat gpurun_out/sd_bench.jsonl
exit $rc
