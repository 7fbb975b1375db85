#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks
# on one device).  The real N>1 runs (RCCL over xGMI, one rank per GPU) are the driver's.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-dist}
mkdir -p "$OUT"
HGIN_DIST_BACKEND=gloo timeout -k 10 ${DIST_TIMEOUT:-400} python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  > "$OUT/bench_2rank_gloo.json" 2> "$OUT/bench_2rank_gloo.err"
echo "dist_rehearsal $?" >> "$OUT/status.txt"
