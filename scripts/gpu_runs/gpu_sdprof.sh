#!/bin/bash
# SDXL 1024^2: denoise-step kernel table + one PMC pass (clock / MFMA busy per kernel),
# and a VAE decode kernel table (no library convolutions expected)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/sdprof; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
echo kt done
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -d $OUT/pmc -o run --output-format csv -- python3 scripts/bench_sd.py --version xl --denoise --graph --steps 3 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
echo pmc done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vae -o run --output-format csv -- python3 scripts/bench_sd.py --version xl --vae > $OUT/vae.log 2>&1 || { tail -20 $OUT/vae.log; exit 1; }
grep '^{' $OUT/vae.log | tail -1 | cut -c1-300
find $OUT -name "*.csv" | head -20
