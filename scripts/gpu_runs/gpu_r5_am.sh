#!/bin/bash
# round 5: GEMM tests after the split-scaling nearest-M rule + the off-grid plan points, then
# 8B TTFT at off-grid prompt lengths: this table vs the previous commit's (engine rebuilt
# with the rule: the old table under the new rule is what "prev" measures) and vs the
# pre-library table
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5am; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [[ $rc -eq 0 ]] || exit $rc
for P in 64 200 700 1500; do
  for T in new old; do
    if [[ $T == old ]]; then export CAKE_GEMM_TABLE=$GRAFT_REPO_ROOT/ab/gemm_tuned_old.json; else unset CAKE_GEMM_TABLE; fi
    timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { tail -20 $OUT/b_${P}_$T.err; exit 1; }
    python -c "
import json; r=json.loads(open('$OUT/b_${P}_$T.json').read().strip().splitlines()[-1]); print(json.dumps({'prompt': $P, 'table': '$T', 'ttft_ms': r['ttft_ms_prefill'], 'decode_tok_s': r['value']}))"
  done
done
