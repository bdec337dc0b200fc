#!/bin/bash
# GPU box, round 5 (k): SDXL denoise step kernel breakdown (rocprofv3 --kernel-trace --stats).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5k; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/bench_sd.py --version xl --denoise --graph --steps 8 > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 1; }
tail -3 $OUT/plain.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/scripts/bench_sd.py" --version xl --denoise --graph --steps 8 > "$ROOT/$OUT/prof.log" 2>&1 || { tail -20 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
cp "$f" "$ROOT/$OUT/kernel_stats.csv"
python3 - "$ROOT/$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot / 1e6, 2))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}')
PY
find "$ROOT/$OUT/prof" -name '*.db' -delete
