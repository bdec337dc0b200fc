#!/bin/bash
# GPU box: 4-stage 160-column GEMM tiles — tests, graph-timed SD re-tune, SDXL step
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/g4; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/before.log 2>&1 || { tail $OUT/before.log; exit 1; }
grep '^{' $OUT/before.log | tail -1 | cut -c1-130
timeout -k 10 500 python scripts/tune_sd_gemm.py --write $OUT/gemm_tuned.json > $OUT/tune.jsonl 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
grep step_gemm $OUT/tune.jsonl
cp $OUT/gemm_tuned.json cake_amd/ops/gemm_tuned.json
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/after.log 2>&1 || { tail $OUT/after.log; exit 1; }
grep '^{' $OUT/after.log | tail -1 | cut -c1-130
timeout -k 10 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8 > $OUT/after15.log 2>&1 || { tail $OUT/after15.log; exit 1; }
grep '^{' $OUT/after15.log | tail -1 | cut -c1-130
