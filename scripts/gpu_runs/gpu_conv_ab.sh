#!/bin/bash
# GPU box: conv epilogue change A/B — previous library (cake_amd/lib/ab/libcake_kernels_old.so)
# vs the in-tree build: conv / SD tests, conv sweep, SDXL and SD1.5 denoise steps.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${CAB_OUT:-cab}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
OLD=$GRAFT_REPO_ROOT/cake_amd/lib/ab/libcake_kernels_old.so
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -5 $OUT/$name.log; exit $rc; }; }
run tests 400 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_sd_gpu.py tests/test_fuzz_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
tail -1 $OUT/tests.log
run sdxl_new 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8
run sdxl_old 300 env CAKE_KERNEL_LIB=$OLD python scripts/bench_sd.py --version xl --denoise --graph --steps 8
run sd15_new 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8
run sd15_old 300 env CAKE_KERNEL_LIB=$OLD python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8
run sdxl_new2 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8
exit 0
