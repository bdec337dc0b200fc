#!/bin/bash
# GPU box, round 5 (ab): native SDXL step kernel tables with the LayerNorm fold on / off.
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5ab; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
cat > $OUT/run_sd.py <<'PY'
import json, sys
sys.path.insert(0, sys.argv[1])
from cake_amd.models.sd.bench import measure_native
print(json.dumps(measure_native("xl", 8, "f16", 0)))
PY
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  CAKE_SD_LN_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof_$f" -o run -- python3 "$ROOT/$OUT/run_sd.py" "$ROOT" > "$ROOT/$OUT/prof_$f.log" 2>&1 || { tail -20 "$ROOT/$OUT/prof_$f.log"; exit 1; }
  DB=$(find "$ROOT/$OUT/prof_$f" -name '*.db' | head -n 1)
  python3 "$ROOT/scripts/kernel_stats_db.py" "$DB" --last-ms 240 --per 8 --top 16 > "$ROOT/$OUT/table_$f.txt"
  echo "=== fold $f"; cat "$ROOT/$OUT/table_$f.txt"
  find "$ROOT/$OUT/prof_$f" -name '*.db' -delete
done
