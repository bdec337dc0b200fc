#!/bin/bash
# GPU box, round 5 (m): SDXL 1024^2 step on the native SD engine vs the Python pipeline.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5m; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python - > $OUT/sd.log 2>&1 <<'PY'
import json
from cake_amd.models.sd.bench import measure_native, measure_denoise
print(json.dumps({"native": measure_native("xl", 8)}), flush=True)
print(json.dumps({"python": measure_denoise("xl", 8)}), flush=True)
print(json.dumps({"native_v15": measure_native("v1-5", 8)}), flush=True)
PY
rc=$?
echo "== rc=$rc"; cat $OUT/sd.log | grep -v amdgpu.ids | cut -c1-700
exit $rc
