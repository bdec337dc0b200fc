#!/bin/bash
# round 6: PMC of the four-wave GEMMs (cfg 22, deep twin 25) against hipBLASLt at 8192^3:
# clock, MFMA busy, wait split, LDS traffic / conflicts
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6l; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
for cfg in 22 25 -1; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/kt_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py 8192 8192 8192 $cfg 20 > $OUT/kt_$cfg.log 2>&1 || exit $?
  for p in 1 2 3; do
    eval "ctr=\$P$p"
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT/p${p}_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py 8192 8192 8192 $cfg 5 > $OUT/p${p}_$cfg.log 2>&1 || exit $?
  done
  echo "cfg $cfg done"
done
exit 0
