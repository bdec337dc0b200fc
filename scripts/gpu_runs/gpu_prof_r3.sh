#!/bin/bash
# GPU box: rocprofv3 kernel traces from HEAD -> per-kernel tables under gpurun_out/proftab/.
#   decode 8B at a 32-token and a 2048-token prompt (scripts/decode_kernel_table.py) and the
#   SDXL 1024^2 denoise step (scripts/prof_window.py, last 5 steps of 8).
# Each rocprofv3 run has its own time limit; the script stops at the first failure.
set -u
ROOT="$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/proftab"
cd /tmp && export TMPDIR=/tmp
db_of() { find "$1" -name '*.db' | head -n 1; }
for P in ${PROMPTS:-32 2048}; do
  rm -rf "$ROOT/gpurun_out/prof_p$P"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_p$P" -o run -- \
    python3 "$ROOT/bench.py" --no-extras --steps 64 --warmup 4 --prompt-len "$P" \
    > "$ROOT/gpurun_out/prof_p$P.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/prof_p$P.log"; exit 1; }
  grep '^{' "$ROOT/gpurun_out/prof_p$P.log" | cut -c1-160
  python3 "$ROOT/scripts/decode_kernel_table.py" "$(db_of "$ROOT/gpurun_out/prof_p$P")" \
    --ctx $((P + 4 + 32)) > "$ROOT/gpurun_out/proftab/decode8b_p$P.txt" || exit 1
  cat "$ROOT/gpurun_out/proftab/decode8b_p$P.txt"
  python3 "$ROOT/scripts/prof_window.py" "$(db_of "$ROOT/gpurun_out/prof_p$P")" 10 12 \
    > "$ROOT/gpurun_out/proftab/decode8b_p${P}_window.txt" || exit 1
done
if [[ ${DO_70B:-0} == 1 ]]; then
  rm -rf "$ROOT/gpurun_out/prof_70b"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_70b" -o run -- \
    python3 "$ROOT/bench.py" --no-extras --model llama3-70b --steps 24 --warmup 4 \
    > "$ROOT/gpurun_out/prof_70b.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/prof_70b.log"; exit 1; }
  grep '^{' "$ROOT/gpurun_out/prof_70b.log" | cut -c1-160
  python3 "$ROOT/scripts/prof_window.py" "$(db_of "$ROOT/gpurun_out/prof_70b")" 100 12 \
    > "$ROOT/gpurun_out/proftab/decode70b_window.txt" || exit 1
  cat "$ROOT/gpurun_out/proftab/decode70b_window.txt"
fi
if [[ ${DO_SDXL:-1} == 1 ]]; then
  rm -rf "$ROOT/gpurun_out/prof_sdxl"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_sdxl" -o run -- \
    python3 "$ROOT/scripts/bench_sd.py" --version xl --denoise --graph --steps 8 \
    > "$ROOT/gpurun_out/prof_sdxl.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/prof_sdxl.log"; exit 1; }
  tail -2 "$ROOT/gpurun_out/prof_sdxl.log"
  python3 "$ROOT/scripts/prof_window.py" "$(db_of "$ROOT/gpurun_out/prof_sdxl")" 155 30 \
    > "$ROOT/gpurun_out/proftab/sdxl_denoise.txt" || exit 1
  head -12 "$ROOT/gpurun_out/proftab/sdxl_denoise.txt"
fi
# the raw traces are large: keep only the tables and the rocprofv3 stats CSVs
find "$ROOT/gpurun_out" -name '*.db' -delete
exit 0
