#!/bin/bash
# round 6 final: the plan table's MFMA kernels vs hipBLASLt, same box, interleaved rounds
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zj; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python scripts/bench_gemm_pp.py --shapes 8b,70b,sq --ms 512,2048 --arms mfma,lib --rounds 5 > $OUT/arms.log 2>&1 || { tail -30 $OUT/arms.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6zj/arms.log"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(f'{r["shape"]:18s} plan={r["mfma_plan"]} mfma={r["mfma_tflops"]:.0f} lib={r["lib_tflops"]:.0f} ratio={r["mfma_tflops"]/r["lib_tflops"]:.3f}')
PY
