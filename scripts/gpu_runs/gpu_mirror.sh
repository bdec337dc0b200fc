#!/bin/bash
# GPU box: token read-back through the pinned ring (mirror node in each step graph) —
# decode / engine / serving tests, smoke, the driver-flag bench and a kernel window
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/mirror; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run tests 700 python -u -m pytest tests/test_model_gpu.py tests/test_engine_gpu.py tests/test_sampling_gpu.py tests/test_serving_gpu.py tests/test_parity_hf.py -x -q --timeout 120 --timeout-method thread
tail -1 $OUT/tests.log
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras
grep '^{' $OUT/bench.log | cut -c1-160
run bench2 300 python bench.py --gpus 1 --steps 128 --warmup 16 --no-extras
grep '^{' $OUT/bench2.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-extras --steps 64 --warmup 4
python3 scripts/prof_window_csv.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) --ms 10 | head -12
