#!/bin/bash
# round 5: 8B TTFT on the native engine, library-GEMM plan table vs the previous one
# (CAKE_GEMM_TABLE=ab/gemm_tuned_old.json), interleaved; then first-call cost of new M
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ah; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
for P in 128 512 1024 2048 4000; do
  for T in new old; do
    if [[ $T == old ]]; then export CAKE_GEMM_TABLE=$GRAFT_REPO_ROOT/ab/gemm_tuned_old.json; else unset CAKE_GEMM_TABLE; fi
    timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { tail -20 $OUT/b_${P}_$T.err; exit 1; }
    python - $OUT/b_${P}_$T.json $P $T <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"prompt": int(sys.argv[2]), "table": sys.argv[3], "ttft_ms": r["ttft_ms_prefill"], "tok_s": r["value"], "engine": r.get("engine")}))
PY
  done
done
unset CAKE_GEMM_TABLE
timeout -k 10 120 python - <<'PY'
import time, torch
from cake_amd.ops import gemm as G
w = torch.randn(6144, 4096, device="cuda").bfloat16()
for M in (1000, 1001, 1002, 1000):
    x = torch.randn(M, 4096, device="cuda").bfloat16()
    torch.cuda.synchronize(); t = time.perf_counter()
    G.linear(x, w, cfg=G.LIB); torch.cuda.synchronize()
    print(f"M={M} library GEMM call incl. plan build: {(time.perf_counter() - t) * 1e3:.3f} ms")
PY
