#!/bin/bash
# GPU box: why SD's short-K projection GEMMs (SDXL attention-out / FF-out at 1024 tokens,
# CFG batch 2) run at ~200-430 TFLOP/s.  Per config: kernel time, MFMA busy + clock,
# L2 hit rate, fabric bytes; hipBLASLt (cfg -1) alongside.  One counter block per pass.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sdpmc
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
for shape in "2048 1280 1280" "2048 1280 5120" "8192 640 640"; do
  tag=$(echo $shape | tr ' ' x)
  for cfg in ${CFGS:-4 0 7 1 -1}; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $OUT/kt_${tag}_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py $shape $cfg 20 > $OUT/kt_${tag}_$cfg.log 2>&1 || exit $?
    for p in 1 2 3; do
      eval "ctr=\$P$p"
      timeout -s KILL 60 rocprofv3 --pmc $ctr -d $OUT/p${p}_${tag}_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py $shape $cfg 5 > $OUT/p${p}_${tag}_$cfg.log 2>&1 || exit $?
    done
    echo "$tag cfg $cfg done"
  done
done
exit 0
