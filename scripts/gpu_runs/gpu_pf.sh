#!/bin/bash
# decode attention prefetch depth A/B: numerics, then the 8B decode bench at 32 / 2048
# prompt tokens per depth, then a kernel table per depth
set -o pipefail
mkdir -p gpurun_out/pf
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "attn or qkv_attn" > gpurun_out/pf/tests.log 2>&1 || { tail -30 gpurun_out/pf/tests.log; exit 1; }
tail -1 gpurun_out/pf/tests.log
for pl in 32 2048; do
  for pf in 0 1 0 2; do
    CAKE_ATTN_PREFETCH=$pf timeout -k 10 300 python -u bench.py --no-extras --no-sd --steps 128 --warmup 16 --prompt-len $pl \
      > gpurun_out/pf/bench_${pl}_$pf.log 2>&1 || { tail -20 gpurun_out/pf/bench_${pl}_$pf.log; exit 1; }
    echo "prompt=$pl pf=$pf $(grep '^{' gpurun_out/pf/bench_${pl}_$pf.log | tail -1 | cut -c1-120)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for pf in 0; do
  CAKE_ATTN_PREFETCH=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/prof_$pf -o run -- \
    python -u bench.py --no-extras --no-sd --steps 32 --warmup 8 > gpurun_out/pf/prof_$pf.log 2>&1 || exit $?
done
