set -e
run() { timeout -k 10 200 env "$@" python bench.py --steps 256 --warmup 32 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', d['value'], d['ms_per_step'])"; }
run CAKE_FUSED=0
run CAKE_FUSED=1 CAKE_AO_SLEEP=1
run CAKE_FUSED=1 CAKE_AO_SLEEP=4
run CAKE_FUSED=1 CAKE_AO_SLEEP=16
run CAKE_FUSED=1 CAKE_AO_SLEEP=4 CAKE_AO_GRID=256
run CAKE_FUSED=1 CAKE_AO_SLEEP=4 CAKE_AO_GRID=1024
run CAKE_FUSED=2 CAKE_AO_SLEEP=4
