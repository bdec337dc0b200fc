#!/bin/bash
# Round-3 GPU iteration: full GPU tests, the driver bench, decode attention phase clocks,
# SDXL denoise seconds/step and its rocprofv3 kernel table.  Each GPU step has its own
# time limit; the script stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  # pytest rc 1 = failed tests (no crash): report and go on to the measurements
  if [[ $rc -eq 1 && $name == pytest* ]]; then grep -E "^FAILED|passed|failed" "gpurun_out/$name.log" | tail -8; return 0; fi
  if [[ $rc -ne 0 ]]; then echo "$name rc=$rc -> stop"; exit $rc; fi
}
if [[ ${DO_SDRCCL:-${DO_TESTS:-1}} == 1 ]]; then
  step pytest_sdrccl 500 python -u -m pytest tests/test_sd_rccl_gpu.py -v -m gpu --timeout 420 --timeout-method thread
fi
if [[ ${DO_TESTS:-1} == 1 ]]; then
  step pytest 600 python -u -m pytest ${TESTS:-tests} -q -m gpu --timeout 120 --timeout-method thread --ignore=tests/test_sd_rccl_gpu.py
fi
[[ ${DO_BENCH:-1} == 1 ]] && step bench 400 python bench.py ${BENCH_ARGS:-}
[[ ${DO_STAMPS:-0} == 1 ]] && step attn_stamps 240 env MINKS=${MINKS:-64} TKS=${TKS:-57,176,512,1024,2048,4000} python scripts/attn_stamps.py
if [[ ${DO_AB2:-0} == 1 ]]; then  # attention core 2 after the one-round merge
  step ab2_impl2 200 env CAKE_ATTN_IMPL=2 python bench.py --no-extras
  step ab2_p2048_impl2 200 env CAKE_ATTN_IMPL=2 python bench.py --no-extras --prompt-len 2048
  step ab2_p2048_impl1 200 env CAKE_ATTN_IMPL=1 python bench.py --no-extras --prompt-len 2048
fi
if [[ ${DO_AB:-0} == 1 ]]; then  # decode A/B: attention core, long context
  step ab_base 200 python bench.py --no-extras
  step ab_impl2 200 env CAKE_ATTN_IMPL=2 python bench.py --no-extras
  step ab_p2048_impl1 200 env CAKE_ATTN_IMPL=1 python bench.py --no-extras --prompt-len 2048
  step ab_p2048_impl2 200 env CAKE_ATTN_IMPL=2 python bench.py --no-extras --prompt-len 2048
fi
if [[ ${DO_AB3:-0} == 1 ]]; then  # fused greedy head (lm_head+penalty+argmax+finalize), core-2 split target
  step ab3_fused 200 python bench.py --no-extras
  step ab3_unfused 200 env CAKE_FUSED_HEAD=0 python bench.py --no-extras
  step ab3_drv_fused 200 python bench.py --no-extras --steps 20 --warmup 5
  step ab3_drv_unfused 200 env CAKE_FUSED_HEAD=0 python bench.py --no-extras --steps 20 --warmup 5
  for tg in ${AB3_TARGETS:-16 32 64}; do
    step ab3_p2048_t$tg 200 env CAKE_ATTN_TARGET=$tg python bench.py --no-extras --prompt-len 2048
    step ab3_p4000_t$tg 200 env CAKE_ATTN_TARGET=$tg python bench.py --no-extras --prompt-len 4000 --max-seq 8192
  done
fi
if [[ ${DO_AB4:-0} == 1 ]]; then  # fused tail incl. embedding vs four launches + embed; PP2 rehearsal
  step ab4_drv_fused 200 python bench.py --no-extras --steps 20 --warmup 5
  step ab4_drv_unfused 200 env CAKE_FUSED_HEAD=0 python bench.py --no-extras --steps 20 --warmup 5
  step ab4_fused 200 python bench.py --no-extras
  step ab4_unfused 200 env CAKE_FUSED_HEAD=0 python bench.py --no-extras
  step ab4_p2048 200 python bench.py --no-extras --prompt-len 2048
  step ab4_pp2 400 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-extras
fi
if [[ ${DO_MULTI:-0} == 1 ]]; then  # multi-rank rehearsals, ranks sharing the one GPU (plumbing)
  step multi_pp2 500 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5
  step multi_tp2 300 python bench.py --gpus 2 --dist-backend gloo --parallel tp --steps 20 --warmup 5 --no-extras
fi
if [[ ${DO_KAB:-0} == 1 ]]; then  # tokens per graph replay
  step k1 200 python bench.py --no-extras --steps 20 --warmup 5
  step k2 200 python bench.py --no-extras --steps 20 --warmup 4 --steps-per-graph 2
  step k4 200 python bench.py --no-extras --steps 20 --warmup 4 --steps-per-graph 4
  step k1b 200 python bench.py --no-extras --steps 128
  step k4b 200 python bench.py --no-extras --steps 128 --steps-per-graph 4
fi
if [[ ${DO_SD:-0} == 1 ]]; then
  step sd_xl 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8
  step sd_15 200 python scripts/bench_sd.py --version v1-5 --denoise --graph --steps 8
fi
if [[ ${DO_SDPROF:-0} == 1 ]]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/sdprof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/sdprof" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_sd.py" --version xl --denoise --graph --steps 8 > "$GRAFT_REPO_ROOT/gpurun_out/sdprof.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/gpurun_out/sdprof.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
fi
exit 0
