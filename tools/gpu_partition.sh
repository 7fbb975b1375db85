#!/bin/bash
# dst-range partition (connected-graph multi-GPU variant): the 2-rank HIP-path parity tests, the 1-rank cfg3
# bench line of the partitioned step, and a 2-rank gloo rehearsal of bench.py --partition dst-range at cfg2
# (both ranks share the one GPU; gloo stages the all-gathers through the host, so its time is not an xGMI figure).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-partition}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -30 "$OUT/$name.log"; exit $rc ;; esac
}
step pytest_dist 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread
step bench_dst1 400 python bench.py --partition dst-range --no-cpu-baseline
HGIN_DIST_BACKEND=gloo step bench_dst2_gloo 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --config cfg2 \
  --partition dst-range --no-probe
echo done >> "$OUT/status.txt"
tail -3 "$OUT/pytest_dist.log"; tail -1 "$OUT/bench_dst1.log"; tail -1 "$OUT/bench_dst2_gloo.log"
