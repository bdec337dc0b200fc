#!/bin/bash
# kernel table: fused QKV + attention vs the two launches (8B decode, short context)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for on in 0 1; do
  CAKE_QKV_ATTN=$on timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qa2_prof_$on -o run -- \
    python -u bench.py --no-extras --no-sd --steps 32 --warmup 8 > gpurun_out/qa2_bench_$on.log 2>&1 || exit $?
done
find gpurun_out/qa2_prof_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -8 "$f" | cut -c1-220; done
