#!/bin/bash
# round 6: native split UNet (2 / 3 ranks sharing the GPU) vs the single-rank engine;
# MFMA-only re-tune of every prefill shape the library GEMM had; TTFT after
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6f; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run split 400 python -u -m pytest tests/test_sd_split_native_gpu.py -x -v --timeout 300 --timeout-method thread
run pair 200 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "pair or big_tile" --timeout 120 --timeout-method thread
run tune 1000 python scripts/tune_sd_gemm.py --lib-shapes --write $OUT/gemm_tuned.json
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
# TTFT on the native engine: MFMA plans (default) vs the library arm (CAKE_GEMM_LIB=1)
for P in 512 2048 4000; do
  for L in 0 1; do
    CAKE_GEMM_LIB=$L timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b_${P}_$L.json 2> $OUT/b_${P}_$L.err || { tail -20 $OUT/b_${P}_$L.err; exit 1; }
    python - $OUT/b_${P}_$L.json $P $L <<'PY' | tee -a $OUT/ttft.jsonl
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"model": "llama3-8b", "prompt": int(sys.argv[2]), "gemm_lib": int(sys.argv[3]), "ttft_ms": r["ttft_ms_prefill"], "tok_s": r["value"]}))
PY
  done
done
for L in 0 1; do
  CAKE_GEMM_LIB=$L timeout -k 10 400 python bench.py --model llama3-70b --no-extras --no-sd --steps 4 --warmup 1 --prompt-len 2048 > $OUT/b70_$L.json 2> $OUT/b70_$L.err || { tail -20 $OUT/b70_$L.err; exit 1; }
  python - $OUT/b70_$L.json $L <<'PY' | tee -a $OUT/ttft.jsonl
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"model": "llama3-70b", "prompt": 2048, "gemm_lib": int(sys.argv[2]), "ttft_ms": r["ttft_ms_prefill"], "tok_s": r["value"]}))
PY
done
