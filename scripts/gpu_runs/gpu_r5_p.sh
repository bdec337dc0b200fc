#!/bin/bash
# GPU box, round 5 (p): head-parallel short-context decode attention — kernel test, then
# the 8B decode bench A/B over CAKE_ATTN_HEADS (off / waves 1, 2, 4) with token dumps.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5p; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run kt 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode_heads" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/kt.log
for h in 0 256:1 256:2 256:4 0; do
  tag=${h/:/_}
  CAKE_ATTN_HEADS=$h run bench_$tag 300 python bench.py --no-extras --no-sd --dump-tokens $OUT/tok_$tag.json
  grep '^{' $OUT/bench_$tag.log | cut -c1-160
done
python - <<'PY'
import json
o = json.load(open("gpurun_out/r5p/tok_0.json"))
for t in ("256_1", "256_2", "256_4"):
    x = json.load(open(f"gpurun_out/r5p/tok_{t}.json"))
    a, b = (o.get("tokens", o) if isinstance(o, dict) else o), (x.get("tokens", x) if isinstance(x, dict) else x)
    n = sum(1 for i, j in zip(a, b) if i == j)
    print(t, "tokens equal", n, "/", len(a))
PY
