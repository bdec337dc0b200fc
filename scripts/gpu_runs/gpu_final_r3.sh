#!/bin/bash
# GPU box: end-of-round check of HEAD as the driver runs it — the whole GPU suite, the
# default bench line — then the SD flash waves-per-workgroup sweep.  Each step has its own
# time limit; the script stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/final; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -15 $OUT/$name.log; exit $rc; }; }
run pytest 720 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
tail -1 $OUT/pytest.log
run bench 240 python bench.py
grep '^{' $OUT/bench.log | cut -c1-400
run flash 150 python scripts/bench_flash_sd_nw.py
cat $OUT/flash.log
exit 0
