#!/bin/bash
# GPU box, round 5 (e): fused attention + o_proj — kernel tests, the decode paths' tests,
# bench A/B (CAKE_ATTN_OPROJ=0/1), rocprofv3 decode kernel table at p32 / p2048.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5e; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; local t0=$(date +%s); timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc wall=$(( $(date +%s) - t0 ))s"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run kt 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn_oproj or attn_decode or gemv" -x -q --timeout 200 --timeout-method thread
tail -2 $OUT/kt.log
run bench_ao1 300 python bench.py --steps 64 --warmup 8 --no-extras --no-sd
grep '^{' $OUT/bench_ao1.log | cut -c1-330
CAKE_ATTN_OPROJ=0 run bench_ao0 300 python bench.py --steps 64 --warmup 8 --no-extras --no-sd
grep '^{' $OUT/bench_ao0.log | cut -c1-330
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_engine_gpu.py tests/test_sampling_gpu.py -q --timeout 300 --timeout-method thread > $OUT/mt.log 2>&1; echo "== mt rc=$?" # python -u -m pytest tests/test_model_gpu.py tests/test_engine_gpu.py tests/test_sampling_gpu.py -q --timeout 300 --timeout-method thread
tail -3 $OUT/mt.log
cd /tmp && export TMPDIR=/tmp
ROOT="$GRAFT_REPO_ROOT"
for P in 32 2048; do
  rm -rf "$ROOT/$OUT/prof_p$P"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_p$P" -o run -- \
    python3 "$ROOT/bench.py" --no-extras --no-sd --steps 64 --warmup 4 --prompt-len "$P" \
    > "$ROOT/$OUT/prof_p$P.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof_p$P.log"; exit 1; }
  grep '^{' "$ROOT/$OUT/prof_p$P.log" | cut -c1-200
  db=$(find "$ROOT/$OUT/prof_p$P" -name '*.db' | head -n 1)
  python3 "$ROOT/scripts/decode_kernel_table.py" "$db" --ctx $((P + 4 + 32)) > "$ROOT/$OUT/decode8b_p$P.txt" || exit 1
  cat "$ROOT/$OUT/decode8b_p$P.txt"
done
find "$ROOT/$OUT" -name '*.db' -delete
exit 0
