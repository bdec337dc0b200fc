#!/bin/bash
# round 6: four-wave tile in the heuristic planners (untuned shapes): tests + square GEMMs
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zl; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/bench_gemm_pp.py --shapes sq,8b,70b --ms 512,2048 --arms mfma,lib --rounds 5 > $OUT/arms.log 2>&1 || { tail -30 $OUT/arms.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6zl/arms.log"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(f'{r["shape"]:18s} plan={r["mfma_plan"]} mfma={r["mfma_tflops"]:.0f} lib={r["lib_tflops"]:.0f} ratio={r["mfma_tflops"]/r["lib_tflops"]:.3f}')
PY
