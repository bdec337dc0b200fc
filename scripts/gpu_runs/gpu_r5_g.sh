#!/bin/bash
# GPU box, round 5 (g): split-UNet device hops — GPU tests, then the full-size SDXL split at
# N=2 and N=4 on one shared GPU (gloo control, device bulk hops).
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5g; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [[ $rc -eq 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
run tests 400 python -u -m pytest tests/test_sd_split_gpu.py -x -v --timeout 300 --timeout-method thread
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -5
run n2 500 python bench.py --gpus 2 --steps 8 --warmup 3 --dist-backend gloo --extras sd --sd-steps 4 --launch-timeout 450
grep '^{' $OUT/n2.log > $OUT/n2.json; python -c "import json;d=json.load(open('$OUT/n2.json'));print(json.dumps(d['sd']))"
run n4 600 python bench.py --gpus 4 --steps 8 --warmup 3 --dist-backend gloo --extras sd --sd-steps 4 --launch-timeout 550
grep '^{' $OUT/n4.log > $OUT/n4.json; python -c "import json;d=json.load(open('$OUT/n4.json'));print(json.dumps(d['sd']))"
