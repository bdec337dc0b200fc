#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "1 1" "1 0" "2 0"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/mk_stamps.py --model llama3-8b --pos 32 --thin 0 --fly $1 --o-all $2 --out gpurun_out/mk9_f$1_o$2.npy > gpurun_out/mk9_stamps.log 2>&1 || exit $?
  grep '^{' gpurun_out/mk9_stamps.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('fly','o_all','layer_us_median','qkv_walk','o_walk','swiglu_walk','down_walk','attn_chain(qkv_pub_last->o_xready_med)','edge_mid(o_done_last->swi_xready_med)','edge_act(swi_done_last->down_xready_med)','edge_res(down_pub_last->qkv_xready_med)','t_qkv_pub','t_o_xready','t_o_done','t_swi_xready','step_us')})"
done
