#!/bin/bash
# GPU box: TP + GEMM(IL) + worker-graph + sampling tests, GEMM sweep (SD shapes), 1-GPU bench,
# TP plumbing at 8B scale with 2 ranks sharing the GPU (not a perf number).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_sampling_gpu.py -x -v --timeout 170 --timeout-method thread > gpurun_out/r2h_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2h_pytest.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 32 --warmup 4 > gpurun_out/bench_tp2_shared.json 2> gpurun_out/bench_tp2_shared.err || exit $?
cat gpurun_out/bench_tp2_shared.json
timeout -k 10 700 python scripts/bench_gemm.py --cfgs 0,8,1,4,5,11,6,2 > gpurun_out/gemm_il2.jsonl 2> gpurun_out/gemm_il2.err || exit $?
cat gpurun_out/gemm_il2.jsonl
exit 0
