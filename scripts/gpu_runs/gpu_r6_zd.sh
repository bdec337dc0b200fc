#!/bin/bash
# round 6: resid32 residual batched per strip in the wide read-out: numerics, A/B, prefill window
set -u
cd "$GRAFT_REPO_ROOT"; ROOT="$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zd; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python scripts/bench_gemm_pp.py --shapes 8b,70b --ms 2048 --arms mfma,lib > $OUT/arms.log 2>&1 || { tail -30 $OUT/arms.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6zd/arms.log"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(r["shape"], r["mfma_plan"], " ".join(f'{a}={r[a+"_tflops"]:.0f}' for a in ("mfma","lib")))
PY
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/native_prefill.py" --len 2048 --reps 3 > "$ROOT/$OUT/prof.log" 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
DB=$(find "$OUT/prof" -name '*.db' | head -n 1)
python3 scripts/kernel_stats_db.py "$DB" --last-ms 30 --top 8 > $OUT/prefill2048.txt
find $OUT -name '*.db' -delete
cat $OUT/prefill2048.txt
