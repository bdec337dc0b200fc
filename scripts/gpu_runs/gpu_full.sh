#!/bin/bash
# the whole GPU suite as the driver runs it (one process, -x), then smoke()
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/full; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -40 $OUT/$name.log; exit $rc; }; }
run pytest ${1:-1050} python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${2:-}
tail -2 $OUT/pytest.log
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
