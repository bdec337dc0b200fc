#!/bin/bash
# GPU box: one PMC pass over the SDXL denoise step — stall classes and LDS conflicts per kernel
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/sdpmc2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/pmc -o run --output-format csv -- python3 scripts/bench_sd.py --version xl --denoise --graph --steps 3 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
ls $OUT/pmc
