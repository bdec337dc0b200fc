#!/bin/bash
# GPU box: effective clock of the SDXL denoise kernels inside the graph (GRBM_GUI_ACTIVE per
# dispatch / 8 / kernel time) — sustained-load clock vs the isolated-GEMM runs.
set -u
ROOT="$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/sdclk"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d "$ROOT/gpurun_out/sdclk" -o run --output-format csv -- \
  python3 "$ROOT/scripts/bench_sd.py" --version xl --denoise --graph --steps 4 > "$ROOT/gpurun_out/sdclk.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/sdclk.log"; exit 1; }
tail -2 "$ROOT/gpurun_out/sdclk.log"
find "$ROOT/gpurun_out/sdclk" -name '*.csv' | head
exit 0
