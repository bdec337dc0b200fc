#!/bin/bash
# GPU box, round 5 (f): fused attention + o_proj A/B (kernel test, bench, p32 kernel table).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5f; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run kt 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_oproj" -x -q --timeout 200 --timeout-method thread
tail -1 $OUT/kt.log
for ao in 1 0; do CAKE_ATTN_OPROJ=$ao run bench_ao$ao 300 python bench.py --steps 64 --warmup 8 --no-extras --no-sd; grep '^{' $OUT/bench_ao$ao.log | cut -c1-200; done
cd /tmp && export TMPDIR=/tmp; ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_p32" -o run -- python3 "$ROOT/bench.py" --no-extras --no-sd --steps 64 --warmup 4 > "$ROOT/$OUT/prof_p32.log" 2>&1 || exit 1
python3 "$ROOT/scripts/decode_kernel_table.py" "$(find "$ROOT/$OUT/prof_p32" -name '*.db' | head -n 1)" --ctx 68 > "$ROOT/$OUT/decode8b_p32.txt" && cat "$ROOT/$OUT/decode8b_p32.txt"
find "$ROOT/$OUT" -name '*.db' -delete
