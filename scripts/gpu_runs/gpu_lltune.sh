#!/bin/bash
# GPU box: graph-timed GEMM plans for the Llama prefill shapes, TTFT before / after
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/lltune; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/bench_prefill.py --lens 512,2048,4096 > $OUT/before.jsonl 2> $OUT/before.err || { tail $OUT/before.err; exit 1; }
cat $OUT/before.jsonl
timeout -k 10 700 python scripts/tune_sd_gemm.py --versions llama --write $OUT/gemm_tuned.json > $OUT/tune.jsonl 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
grep step_gemm $OUT/tune.jsonl
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
timeout -k 10 200 python scripts/bench_prefill.py --lens 512,2048,4096 > $OUT/after.jsonl 2> $OUT/after.err || { tail $OUT/after.err; exit 1; }
cat $OUT/after.jsonl
