#!/bin/bash
# GPU box: TP tests (2 and 4 ranks sharing the GPU), decode speed-of-light probe,
# TP4 bench rehearsal (4 ranks on one GPU, gloo host collectives), 1-GPU bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2o_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r2o_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A30 "Error\|FAILED" gpurun_out/r2o_pytest.log | head -80; exit $rc; fi
timeout -k 10 300 python scripts/decode_ceiling.py > gpurun_out/ceiling.jsonl 2> gpurun_out/ceiling.err || { tail -20 gpurun_out/ceiling.err; exit 1; }
cat gpurun_out/ceiling.jsonl
timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --steps 64 --warmup 8 > gpurun_out/tp4_shared.json 2> gpurun_out/tp4_shared.err || { tail -20 gpurun_out/tp4_shared.err; exit 1; }
cat gpurun_out/tp4_shared.json
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
exit 0
