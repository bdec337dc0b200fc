#!/bin/bash
# round 6: four-wave epilogue with whole-line stores: numerics, stamps, A/B
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6u; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for s in "8192 8192 8192" "4096 4096 4096" "2048 8192 28672"; do
  timeout -k 10 60 ./scripts/gemm_stamp $s | tee -a $OUT/stamps.jsonl || exit 1
done
timeout -k 10 500 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 2048 --arms mfma,w4,b4,w3,b3,w1,b1,lib > $OUT/arms.log 2>&1 || { tail -30 $OUT/arms.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6u/arms.log"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(r["shape"], " ".join(f'{a}={r[a+"_tflops"]:.0f}' for a in ("mfma","w4","b4","w3","b3","w1","b1","lib")), "maxerr", max(v for k, v in r.items() if k.endswith("_err")))
PY
