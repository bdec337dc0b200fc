#!/bin/bash
# GPU box: PMC of the interleaved 256x256 GEMM tile vs hipBLASLt at 8192^3 (stall split).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc2
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL"
for cfg in 5 0 -1; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc2/p1_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py 8192 8192 8192 $cfg 5 > gpurun_out/pmc2/p1_$cfg.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc2/p2_$cfg -o run --output-format csv -- python3 scripts/gemm_pmc.py 8192 8192 8192 $cfg 5 > gpurun_out/pmc2/p2_$cfg.log 2>&1 || exit $?
  echo "cfg $cfg done"
done
timeout -k 10 200 python scripts/bench_sd.py --version xl --vae --steps 3 > gpurun_out/vae.json 2> gpurun_out/vae.err || exit $?
timeout -k 10 200 python scripts/bench_sd.py --version v1-5 --vae --steps 3 >> gpurun_out/vae.json 2>> gpurun_out/vae.err || exit $?
cat gpurun_out/vae.json
