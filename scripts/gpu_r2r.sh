#!/bin/bash
# GPU box: kernels / model / TP tests with the split-prologue GEMV defaults, 1-GPU bench,
# decode kernel traces at prompt 32 and 2048 (per-kernel bytes / TB/s tables).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 800 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_tp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2r_pytest.log
if [[ $rc -ne 0 ]]; then grep -B2 -A30 "Error\|FAILED" gpurun_out/r2r_pytest.log | head -80; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r2r.json 2> gpurun_out/bench_r2r.err || { tail gpurun_out/bench_r2r.err; exit 1; }
cat gpurun_out/bench_r2r.json
cd /tmp && export TMPDIR=/tmp
for P in 32 2048; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2r_$P" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --prompt-len $P --steps 32 --warmup 4 --max-seq 4096 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r2r_$P.log" 2>&1 || exit $?
done
cd "$GRAFT_REPO_ROOT"
python scripts/decode_kernel_table.py gpurun_out/prof_r2r_32/run_results.db --ctx 55
python scripts/decode_kernel_table.py gpurun_out/prof_r2r_2048/run_results.db --ctx 2071
exit 0
