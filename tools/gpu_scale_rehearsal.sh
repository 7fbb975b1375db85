#!/bin/bash
# 2-rank rehearsal (gloo, both ranks on the one GPU) of bench.py's default N > 1 path: cfg4's components split,
# plus rank 0's in-run single-GPU reference of all 8 components (scaling_vs_1gpu).  The real N > 1 runs (RCCL,
# one rank per GPU) are the driver's; two ranks sharing one GPU make the N = 2 time and ratio meaningless as
# scaling figures — this checks the flow end to end.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-scale_rehearsal}
mkdir -p "$OUT"
export TMPDIR=/tmp
HGIN_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-probe \
  > "$OUT/bench_2rank.json" 2> "$OUT/bench_2rank.err"
rc=$?; echo "bench_2rank $rc" >> "$OUT/status.txt"
tail -1 "$OUT/bench_2rank.json"; exit $rc
