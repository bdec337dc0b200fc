#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "
import json
from cake_amd.models.sd.bench import measure_native
r = measure_native('xl', 8)
print(json.dumps({k: r[k] for k in ('seconds_per_step', 'text_ms', 'vae_decode_ms', 'image_wall_s')}))
" > gpurun_out/r5_as.json 2> gpurun_out/r5_as.err || { tail -20 gpurun_out/r5_as.err; exit 1; }
cat gpurun_out/r5_as.json
