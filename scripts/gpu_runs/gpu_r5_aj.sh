#!/bin/bash
# round 5: 8B prefill kernel table at 2048 tokens with the library-GEMM plans (rocprofv3
# kernel trace of bench_prefill.py), then 70B TTFT new vs old plan table (native engine)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5aj; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/bench_prefill.py" --lens 2048 --reps 3 > "$ROOT/$OUT/prof.log" 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
DB=$(find "$OUT/prof" -name '*.db' | head -n 1)
python3 scripts/kernel_stats_db.py "$DB" --last-ms 29 --top 25 > $OUT/prefill2048.txt
cat $OUT/prefill2048.txt
find $OUT -name '*.db' -delete
for P in 512 2048; do
  for T in new old; do
    if [[ $T == old ]]; then export CAKE_GEMM_TABLE=$ROOT/ab/gemm_tuned_old.json; else unset CAKE_GEMM_TABLE; fi
    timeout -k 10 400 python bench.py --model llama3-70b --no-extras --no-sd --steps 4 --warmup 1 --prompt-len $P > $OUT/b70_${P}_$T.json 2> $OUT/b70_${P}_$T.err || { tail -20 $OUT/b70_${P}_$T.err; exit 1; }
    python -c "
import json; r=json.loads(open('$OUT/b70_${P}_$T.json').read().strip().splitlines()[-1]); print(json.dumps({'model': '70b', 'prompt': $P, 'table': '$T', 'ttft_ms': r['ttft_ms_prefill'], 'decode_tok_s': r['value']}))"
  done
done
