#!/bin/bash
# round 5: hipBLASLt warm-up at engine open: engine tests, then the FIRST request's prefill
# time at 2048 tokens (before: ~175 ms of library init on top; the bench's TTFT is warm)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r5_ay.log 2>&1
rc=$?; tail -2 gpurun_out/r5_ay.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 200 python - <<'PY'
import time, torch
from cake_amd.engine import NativeLlama
from cake_amd.parallel.native_bench import _config_dir
from cake_amd.models.llama3.config import preset
cfg = preset("llama3-8b")
torch.cuda.set_device(0)
t0 = time.time()
eng = NativeLlama(_config_dir(cfg), max_seq=2304, dtype="bf16", device=0, random_init=True, seed=1)
print(f"open {time.time() - t0:.2f} s")
prompt = [int(x) for x in torch.randint(0, cfg.vocab_size, (2048,))]
for i in range(2):
    r = eng.generate(prompt, 2, temperature=0.0, eos_ids=[])
    print(f"request {i}: prefill {r.prefill_s * 1e3:.1f} ms")
eng.close()
PY
