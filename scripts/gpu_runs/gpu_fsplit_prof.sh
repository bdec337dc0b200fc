#!/bin/bash
# GPU box: kernel times of the flash key split (split kernel vs merge launch) at SD shapes
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/fsprof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 scripts/bench_flash_split.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("gpurun_out/fsprof/kt/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: [0, 0])
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "flash" not in n: continue
    k = (n.split("(")[0][-40:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[k][0] += 1; agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, (c, t) in sorted(agg.items()):
    print(k, c, round(t / c / 1e3, 2), "us")
PY
