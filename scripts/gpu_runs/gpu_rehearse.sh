#!/bin/bash
# Shared-GPU rehearsal of the multi-rank bench: N ranks (torchrun, one process per rank)
# all on this box's one GPU — the full default bench (8B pp / tp / pp_streams, 70B pp / tp,
# the split-UNet SDXL sub-record).  Numbers are time-sharing artefacts; the point is that
# every sub-record runs, its wall time, and per-rank HBM (host collectives on gloo: RCCL
# refuses two ranks on one GPU; the in-graph hops / all-reduces are the device IPC ones).
# usage: gpu_rehearse.sh N [timeout_s]
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/rehearse; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
N=${1:-2}
(while sleep 50; do date >> $OUT/heartbeat_n$N; done) & HB=$!
start=$(date +%s)
timeout -k 10 ${2:-1050} python -m torch.distributed.run --nnodes 1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 20 --warmup 5 --dist-backend gloo \
  > $OUT/bench_n$N.log 2>&1
rc=$?
end=$(date +%s)
kill $HB 2>/dev/null
echo "rc=$rc wall_s=$((end - start))" | tee $OUT/wall_n$N.txt
grep '^{' $OUT/bench_n$N.log | tail -1 > $OUT/bench_n$N.json || true
cut -c1-1500 $OUT/bench_n$N.json
[[ $rc -eq 0 ]] || tail -30 $OUT/bench_n$N.log
exit $rc
