set -e
for k in 1 2 4 8 1; do
  timeout -k 10 200 python bench.py --steps 256 --warmup 32 --steps-per-graph $k 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('k=$k', d['value'], d['ms_per_step'], d['p50_token_latency_ms'], d['p99_token_latency_ms'])"
done
