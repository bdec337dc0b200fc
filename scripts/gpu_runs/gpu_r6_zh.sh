#!/bin/bash
# round 6 records: default bench on the final plan table, 8B TTFT + decode vs prompt length,
# 70B TTFT at 512 / 2048 (native engine, MFMA-only GEMMs)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zh; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
for P in 128 512 1024 2048 4096 8000; do
  timeout -k 10 300 python bench.py --no-extras --no-sd --steps 64 --warmup 4 --prompt-len $P --max-seq 8192 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(json.dumps({'model': 'llama3-8b', 'prompt': $P, 'ttft_ms': r['ttft_ms_prefill'], 'decode_tok_s': r['value']}))" | tee -a $OUT/sweep.jsonl
done
for P in 512 2048; do
  timeout -k 10 400 python bench.py --model llama3-70b --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b70.json 2> $OUT/b70.err || { tail -20 $OUT/b70.err; exit 1; }
  python -c "import json; r=json.loads(open('$OUT/b70.json').read().strip().splitlines()[-1]); print(json.dumps({'model': 'llama3-70b', 'prompt': $P, 'ttft_ms': r['ttft_ms_prefill'], 'decode_tok_s': r['value']}))" | tee -a $OUT/sweep.jsonl
done
