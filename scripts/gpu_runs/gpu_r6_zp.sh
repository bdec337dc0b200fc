#!/bin/bash
# round 6: N=4 rehearsal with the ranks sharing one GPU (not a scaling number): every
# sub-record on the final tree
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6zp; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 1000 python bench.py --gpus 4 --dist-backend gloo --launch-timeout 900 > $OUT/n4.log 2>&1 || { tail -30 $OUT/n4.log; exit 1; }
grep '^{' $OUT/n4.log | tail -1 | cut -c1-400
