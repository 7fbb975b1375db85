#!/bin/bash
# Final-tree lines for the non-headline workloads: cfg5 (bf16), cfg4 on one GPU (8 components), Zipf(1.1)
# destinations, and the 1-rank dst-range partitioned step.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-other_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -30 "$OUT/$name.log"; exit $rc ;; esac
}
step cfg5 400 python bench.py --config cfg5 --no-cpu-baseline
step cfg4 400 python bench.py --config cfg4 --no-cpu-baseline --no-extras
step zipf 500 python bench.py --skew zipf --no-cpu-baseline --no-extras
step dst1 400 python bench.py --partition dst-range --no-cpu-baseline
echo done >> "$OUT/status.txt"
