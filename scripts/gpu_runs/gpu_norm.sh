#!/bin/bash
# GPU box: norm kernel changes — tests, SDXL / SD1.5 steps, then a kernel trace of the SDXL step
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/norm; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_sd_kernels_gpu.py tests/test_sd_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm or layer or group or unet or denoise" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/xl.log 2>&1 || { tail $OUT/xl.log; exit 1; }
grep '^{' $OUT/xl.log | tail -1 | cut -c1-150
timeout -k 10 300 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8 > $OUT/v15.log 2>&1 || { tail $OUT/v15.log; exit 1; }
grep '^{' $OUT/v15.log | tail -1 | cut -c1-150
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 scripts/prof_window_csv.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) --ms 148 | grep -i "norm\|window"
