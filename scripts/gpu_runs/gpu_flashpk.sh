#!/bin/bash
# GPU box: packed softmax arithmetic in flash v2 — tests, SD shape timing, SDXL step, then
# one PMC pass (stall classes) over the SDXL step
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/flashpk; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or prefill" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 200 python scripts/bench_flash_split.py > $OUT/split.jsonl 2> $OUT/split.err || { tail $OUT/split.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/split.jsonl'):
    d=json.loads(l); print(d['shape'], 'auto', d['ks0_us'], 'us', d['ks0_tflops'], 'TF/s')"
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/xl.log 2>&1 || { tail $OUT/xl.log; exit 1; }
grep '^{' $OUT/xl.log | tail -1 | cut -c1-130
timeout -k 10 200 python scripts/bench_prefill.py --lens 2048,4096 > $OUT/prefill.jsonl 2>&1 || { tail $OUT/prefill.jsonl; exit 1; }
cat $OUT/prefill.jsonl
bash scripts/gpu_sdpmc2.sh && python3 scripts/prof_pmc_stalls.py gpurun_out/sdpmc2/pmc/run_counter_collection.csv --last 1932 | grep -i "flash\|kernel "
