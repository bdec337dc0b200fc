#!/bin/bash
# GPU box: the large-GEMM gap to hipBLASLt (8192^3 and the 8B gate|up shape at 2048 tokens):
# kernel time + MFMA busy / wait split + LDS bank conflicts + L2 hit / fabric bytes per config.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bigpmc
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum"
for shape in "8192 8192 8192" "2048 28672 4096"; do
  tag=$(echo $shape | tr ' ' x)
  for cfg in ${CFGS:-5 0 -1}; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/kt_${tag}_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py $shape $cfg 20 > $OUT/kt_${tag}_$cfg.log 2>&1 || exit $?
    for p in 1 2 3; do
      eval "ctr=\$P$p"
      timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT/p${p}_${tag}_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py $shape $cfg 5 > $OUT/p${p}_${tag}_$cfg.log 2>&1 || exit $?
    done
    echo "$tag cfg $cfg done"
  done
done
exit 0
