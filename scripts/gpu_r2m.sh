#!/bin/bash
# GPU box: TP tests with the GEMV-epilogue push, TP2 (shared GPU) bench push vs no push.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r2m_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2m_pytest.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 64 --warmup 8 > gpurun_out/tp2_push.json 2> gpurun_out/tp2_push.err || exit $?
CAKE_TP_PUSH=0 timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 64 --warmup 8 > gpurun_out/tp2_nopush.json 2> gpurun_out/tp2_nopush.err || exit $?
cat gpurun_out/tp2_push.json gpurun_out/tp2_nopush.json
exit 0
