#!/bin/bash
# GPU-box check of the one-launch QKV+attention decode path: numerics tests, then
# 8B decode tok/s with it off (MAX_T=0) / on, at several context lengths (crossover).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "qkv or decoder or pipeline" --timeout 120 --timeout-method thread > gpurun_out/qa_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/qa_pytest.log
if [[ $rc -ne 0 ]]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
out=gpurun_out/qkv_attn_sweep.txt
echo "# Llama-3-8B decode on 1x MI355X: prompt_len, CAKE_QKV_ATTN_MAX_T, tok/s, ms/step" > $out
for P in ${PROMPTS:-32 512 1024 2048}; do
  for T in 0 100000; do
    CAKE_QKV_ATTN_MAX_T=$T timeout -k 10 240 python bench.py --prompt-len $P --steps 64 --warmup 8 > gpurun_out/qa_${P}_${T}.json 2> gpurun_out/qa_${P}_$T.err
    b=$?
    if [[ $b -ne 0 ]]; then echo "P=$P T=$T bench rc=$b -> stop"; tail -5 gpurun_out/qa_${P}_$T.err; exit $b; fi
    python -c "import json; d=json.load(open('gpurun_out/qa_${P}_${T}.json')); print($P, $T, d['value'], d['ms_per_step'])" >> $out
  done
done
cat $out
