#!/bin/bash
# round end: 8B decode tok/s and TTFT vs context length (native engine, 64 timed steps)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5av; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
for P in 32 512 2048 4096 8000; do
  timeout -k 10 240 python bench.py --no-extras --no-sd --steps 64 --warmup 8 --prompt-len $P --max-seq 8192 > $OUT/b_$P.json 2> $OUT/b_$P.err || { tail -20 $OUT/b_$P.err; exit 1; }
  python -c "
import json; r=json.loads(open('$OUT/b_$P.json').read().strip().splitlines()[-1]); print(json.dumps({'prompt': $P, 'tok_s': r['value'], 'p50_ms': r['p50_token_latency_ms'], 'ttft_ms': r['ttft_ms_prefill'], 'engine': r.get('engine')}))"
done
