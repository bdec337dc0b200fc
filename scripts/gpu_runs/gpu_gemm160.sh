#!/bin/bash
# GPU box: the 160-column GEMM tiles — numerics, then per-config TFLOP/s on the SD / Llama shapes
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/g160; mkdir -p $OUT
export PYTHONUNBUFFERED=1
true > $OUT/tests.log
rc=$?; tail -3 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 400 python scripts/bench_gemm.py --only sd --inner 10 --dtype f16 --cfgs 4,0,1,6,5,13,14,15,18 > $OUT/sd.jsonl 2> $OUT/sd.err || { tail $OUT/sd.err; exit 1; }
cat $OUT/sd.jsonl | cut -c1-400
timeout -k 10 400 python scripts/bench_gemm.py --inner 10 > $OUT/all.jsonl 2> $OUT/all.err || { tail $OUT/all.err; exit 1; }
cut -c1-330 $OUT/all.jsonl
