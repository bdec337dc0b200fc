#!/bin/bash
# round 6: A/B in one call -- wide read-out on every tile shape (this tree) vs only on the
# 64 / 128-column tiles (ab_prev/, the previous commit): SDXL step and 8B TTFT, alternated
set -u
cd "$GRAFT_REPO_ROOT"; ROOT="$GRAFT_REPO_ROOT"; OUT=$ROOT/gpurun_out/r6zc; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
SD='import json; from cake_amd.models.sd.bench import measure_native as m; r = m("xl", 8); print(json.dumps({"sdxl_s": r["seconds_per_step"]}))'
for rep in 1 2; do
  for T in new prev; do
    D=$ROOT; [[ $T == prev ]] && D=$ROOT/ab_prev
    ( cd $D && timeout -k 10 300 python -c "$SD" > $OUT/sd_$T.log 2>&1 ) || { tail -20 $OUT/sd_$T.log; exit 1; }
    echo "$T $(tail -1 $OUT/sd_$T.log)"
    for P in 512 2048; do
      ( cd $D && timeout -k 10 240 python bench.py --no-extras --no-sd --steps 8 --warmup 2 --prompt-len $P > $OUT/b.json 2> $OUT/b.err ) || { tail -20 $OUT/b.err; exit 1; }
      python -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$T', $P, r['ttft_ms_prefill'])"
    done
  done
done
