#!/bin/bash
# GPU box: SD projection shapes in isolation, f16 + add16 (as in the UNet) vs bf16 + store
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/epi; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for shape in "2048 1280 1280" "2048 1280 5120"; do
  for v in "f16 add16" "bf16 store" "f16 store"; do
    tag=$(echo $shape $v | tr ' ' _)
    timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- python3 scripts/gemm_epi_probe.py $shape 4 $v 20 > $OUT/$tag.log 2>&1 || exit $?
    python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')))
rows=[r for r in rows if 'gemm' in r['Name']]
print('$tag', [(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in rows])"
  done
done
