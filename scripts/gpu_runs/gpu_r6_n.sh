#!/bin/bash
# round 6: three-barrier schedule placements (S1 = cfg 25/27, S2 = 28/30, S3 = 29/31) A/B
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6n; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 2048 --arms w4,b4,c4,e4,w1,b1,c1,e1,lib > $OUT/arms.log 2>&1 || { tail -30 $OUT/arms.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6n/arms.log"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(r["shape"], " ".join(f'{a}={r[a+"_tflops"]:.0f}' for a in ("w4","b4","c4","e4","w1","b1","c1","e1","lib")), "maxerr", max(v for k, v in r.items() if k.endswith("_err")))
PY
