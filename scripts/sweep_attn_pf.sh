#!/bin/bash
# GPU-box sweep: decode attention's Infinity-Cache warm-up of wo (CAKE_ATTN_PF_ROWS extra grid rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/attn_pf_sweep.txt
echo "# 8B decode, bench.py ${BENCH_ARGS:-} (tok/s ms/step) per CAKE_ATTN_PF_ROWS" > $out
for r in ${ROWS:-0 8 16 32 64 0}; do
  CAKE_ATTN_PF_ROWS=$r timeout -k 10 240 python bench.py ${BENCH_ARGS:-} > gpurun_out/pf_$r.json 2> gpurun_out/pf_$r.err
  b=$?
  if [[ $b -ne 0 ]]; then echo "rows=$r bench rc=$b -> stop"; tail -5 gpurun_out/pf_$r.err; exit $b; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/pf_$r.json')); print('CAKE_ATTN_PF_ROWS=$r', d['value'], d['ms_per_step'])" >> $out
done
cat $out
