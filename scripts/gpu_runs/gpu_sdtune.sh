#!/bin/bash
# GPU box: measured GEMM plans for the UNet step's exact shapes, then the SDXL step with them
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/sdtune; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python scripts/tune_sd_gemm.py --write $OUT/gemm_tuned.json > $OUT/tune.jsonl 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
grep step_gemm $OUT/tune.jsonl
true
true
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/after.log 2>&1 || { tail $OUT/after.log; exit 1; }
grep '^{' $OUT/after.log | tail -1 | cut -c1-200
timeout -k 10 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8 > $OUT/after15.log 2>&1 || { tail $OUT/after15.log; exit 1; }
grep '^{' $OUT/after15.log | tail -1 | cut -c1-200
