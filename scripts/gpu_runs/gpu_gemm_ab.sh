#!/bin/bash
# GPU box: GEMM epilogue change A/B — old kernel library (cake_amd/lib/ab/libcake_kernels_old.so,
# CAKE_KERNEL_LIB) vs the in-tree build: GEMM tests, per-shape sweep, SDXL step, TTFT.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${GAB_OUT:-gab}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
OLD=$GRAFT_REPO_ROOT/cake_amd/lib/ab/libcake_kernels_old.so
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -5 $OUT/$name.log; exit $rc; }; }
run tests 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_sd_kernels_gpu.py tests/test_sd_gpu.py tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
tail -1 $OUT/tests.log
run gemm_new 300 python scripts/bench_gemm.py
run gemm_old 300 env CAKE_KERNEL_LIB=$OLD python scripts/bench_gemm.py
run sd_new 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8
run sd_old 300 env CAKE_KERNEL_LIB=$OLD python scripts/bench_sd.py --version xl --denoise --graph --steps 8
run ttft_new 200 python bench.py --no-extras --prompt-len 2048 --steps 8 --warmup 2
run ttft_old 200 env CAKE_KERNEL_LIB=$OLD python bench.py --no-extras --prompt-len 2048 --steps 8 --warmup 2
exit 0
