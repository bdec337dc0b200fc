#!/bin/bash
# GPU box iteration: selected tests, 1-GPU bench (default + extra configs), rocprofv3
# kernel profile + per-kernel decode table.  Every GPU step has its own time limit and
# the script stops at the first failure.
#   TESTS="tests/test_kernels_gpu.py ..."  EXTRA="--prompt-len 2048;..."  PROF=1
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [[ -n "${TESTS:-}" ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/iter_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/iter_pytest.log
  if [[ $rc -ne 0 ]]; then grep -A25 "FAILED\|Error" gpurun_out/iter_pytest.log | head -60; exit $rc; fi
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/iter_bench$i.json 2> gpurun_out/iter_bench$i.err || { tail gpurun_out/iter_bench$i.err; exit 1; }
  cat gpurun_out/iter_bench$i.json
done
IFS=';' read -ra XB <<< "${EXTRA:-}"
j=0
for args in "${XB[@]}"; do
  j=$((j+1))
  timeout -k 10 300 python bench.py $args > gpurun_out/iter_x$j.json 2> gpurun_out/iter_x$j.err || { echo "[$args]"; tail gpurun_out/iter_x$j.err; exit 1; }
  echo "[$args]"; cat gpurun_out/iter_x$j.json
done
if [[ -n "${PROF:-}" ]]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/iprof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/iprof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 4 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/iprof.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/gpurun_out/iprof.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  python scripts/decode_kernel_table.py gpurun_out/iprof/run_results.db --ctx 66
fi
exit 0
