#!/bin/bash
# GPU-box check: tests, then the 1-GPU bench, then a rocprofv3 kernel profile.
# Stops at the first fault/abort/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-tests,bench,prof}
rc=0
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest.log
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  b=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  if [[ $b -ne 0 ]]; then echo "bench rc=$b -> stop"; exit $b; fi
fi
if [[ $STEPS == *extra* ]]; then
  # EXTRA_BENCH="args one;args two": further bench configurations, one line each
  IFS=';' read -ra XB <<< "${EXTRA_BENCH:-}"
  i=0
  for args in "${XB[@]}"; do
    i=$((i+1))
    timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > gpurun_out/bench_x$i.json 2> gpurun_out/bench_x$i.err
    b=$?; echo "[$args]"; cat gpurun_out/bench_x$i.json; tail -2 gpurun_out/bench_x$i.err
    if [[ $b -ne 0 ]]; then echo "bench rc=$b -> stop"; exit $b; fi
  done
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 4 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  p=$?; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
  if [[ $p -ne 0 ]]; then echo "prof rc=$p"; exit $p; fi
fi
exit $rc
