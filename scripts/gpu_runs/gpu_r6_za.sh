#!/bin/bash
# round 6: re-tune (Llama prefill shapes + SDXL step shapes) after the wide epilogue read-out in every kernel
# change; TTFT MFMA vs library arm; SDXL step
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6za; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run tune 700 python scripts/tune_sd_gemm.py --lib-shapes --write $OUT/gemm_tuned.json
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
run tunesd 600 python scripts/tune_sd_gemm.py --versions xl --write $OUT/gemm_tuned.json
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
SD='import json; from cake_amd.models.sd.bench import measure_native as m; r = m("xl", 8); print(json.dumps({k: r[k] for k in ("seconds_per_step", "per_step_s")}))'
run sdxl 300 python -c "$SD"
for P in 512 2048; do
  for L in 0 1 0 1; do
    CAKE_GEMM_LIB=$L timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python - $OUT/b.json $P $L <<'PY' | tee -a $OUT/ttft.jsonl
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"model": "llama3-8b", "prompt": int(sys.argv[2]), "gemm_lib": int(sys.argv[3]), "ttft_ms": r["ttft_ms_prefill"], "tok_s": r["value"]}))
PY
  done
done
for L in 0 1; do
  CAKE_GEMM_LIB=$L timeout -k 10 400 python bench.py --model llama3-70b --no-extras --no-sd --steps 4 --warmup 1 --prompt-len 2048 > $OUT/b70.json 2> $OUT/b70.err || { tail -20 $OUT/b70.err; exit 1; }
  python - $OUT/b70.json $L <<'PY' | tee -a $OUT/ttft.jsonl
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"model": "llama3-70b", "prompt": 2048, "gemm_lib": int(sys.argv[2]), "ttft_ms": r["ttft_ms_prefill"], "tok_s": r["value"]}))
PY
done
