#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "0 0 0" "0 0 1" "0 0 2" "1 0 1" "0 0 3"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin $1 --ring $2 --fly $3 > gpurun_out/mk8_stamps.log 2>&1 || exit $?
  grep '^{' gpurun_out/mk8_stamps.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('thin','ring','fly','layer_us_median','qkv_walk','o_walk','swiglu_walk','down_walk','attn_chain(qkv_pub_last->o_xready_med)','edge_mid(o_done_last->swi_xready_med)','edge_act(swi_done_last->down_xready_med)','edge_res(down_pub_last->qkv_xready_med)','step_us')})"
done
