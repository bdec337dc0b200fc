#!/bin/bash
# round 6 final: the whole GPU suite as the driver runs it, smoke, the default bench, the
# 8B prefill kernel table at 2048 tokens (no library GEMM), the N=2 shared-GPU rehearsal
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6final4; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $OUT/$name.log; [[ $rc -eq 0 ]] || { tail -60 $OUT/$name.log; exit $rc; }; }
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
cp $OUT/bench.log $OUT/bench_1gpu.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/native_prefill.py" --len 2048 --reps 3 > "$ROOT/$OUT/prof.log" 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
DB=$(find "$OUT/prof" -name '*.db' | head -n 1)
python3 scripts/kernel_stats_db.py "$DB" --last-ms 30 --top 25 > $OUT/prefill2048.txt
cat $OUT/prefill2048.txt | head -20
find $OUT -name '*.db' -delete
( cd /tmp && export TMPDIR=/tmp && CAKE_GEMM_LIB=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/proflib" -o run -- python3 "$ROOT/scripts/native_prefill.py" --len 2048 --reps 3 > "$ROOT/$OUT/proflib.log" 2>&1 ) || { tail -20 $OUT/proflib.log; exit 1; }
DB=$(find "$OUT/proflib" -name '*.db' | head -n 1)
python3 scripts/kernel_stats_db.py "$DB" --last-ms 30 --top 25 > $OUT/prefill2048_lib.txt
find $OUT -name '*.db' -delete
run n2 900 python bench.py --gpus 2 --dist-backend gloo --launch-timeout 600
