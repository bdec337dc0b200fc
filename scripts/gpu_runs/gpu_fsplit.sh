#!/bin/bash
# GPU box: flash key split — tests, SD shape timing per split count, SDXL / SD1.5 step
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/fsplit; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_sd_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 200 python scripts/bench_flash_split.py > $OUT/split.jsonl 2> $OUT/split.err || { tail $OUT/split.err; exit 1; }
cat $OUT/split.jsonl
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/xl.log 2>&1 || { tail $OUT/xl.log; exit 1; }
grep '^{' $OUT/xl.log | tail -1 | cut -c1-150
true
true
timeout -k 10 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8 > $OUT/v15.log 2>&1 || { tail $OUT/v15.log; exit 1; }
grep '^{' $OUT/v15.log | tail -1 | cut -c1-150
