#!/bin/bash
# GPU box: full GPU suite, smoke(), 1-GPU bench, TP2 rehearsal (2 ranks share the GPU).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2t_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A30 "Error\|FAILED" gpurun_out/r2t_pytest.log | head -80; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r2t.json 2> gpurun_out/bench_r2t.err || { tail gpurun_out/bench_r2t.err; exit 1; }
cat gpurun_out/bench_r2t.json
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 64 --warmup 8 > gpurun_out/tp2_r2t.json 2> gpurun_out/tp2_r2t.err || { tail gpurun_out/tp2_r2t.err; exit 1; }
cat gpurun_out/tp2_r2t.json
exit 0
