#!/bin/bash
# GPU box, round 5 (j): TTFT at short prompts — tune the 8B prefill GEMM plans at 256 / 384 /
# 768 / 1536 rows (the 256-row shapes had no plan: TTFT(256) > TTFT(512)), before/after bench.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5j; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
for P in 256 512; do run before_$P 200 python bench.py --no-extras --no-sd --steps 16 --warmup 4 --prompt-len $P; grep '^{' $OUT/before_$P.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print($P, d['value'], d['ttft_ms_prefill'])"; done
run tune 500 python scripts/tune_sd_gemm.py --versions llama --llama-lens "8b:256,384,768,1536;70b:256" --write cake_amd/ops/gemm_tuned.json
cp cake_amd/ops/gemm_tuned.json $OUT/gemm_tuned.json; cp $OUT/tune.log $OUT/tune.jsonl
for P in 256 384 512 768 1536; do run after_$P 200 python bench.py --no-extras --no-sd --steps 16 --warmup 4 --prompt-len $P; grep '^{' $OUT/after_$P.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print($P, d['value'], d['ttft_ms_prefill'])"; done
