#!/bin/bash
# cfg3 (10M nodes / 100M edges, H=256, L=3) on one MI355X + a pruned-dead-relations cfg2 line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-cfg3}
mkdir -p "$OUT"
timeout -k 10 ${T3:-900} python bench.py --config cfg3 --steps 3 --warmup 1 > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err"
rc=$?; echo "cfg3 $rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --prune-dead --no-cpu-baseline > "$OUT/bench_cfg2_pruned.json" 2> "$OUT/bench_cfg2_pruned.err"
echo "cfg2_pruned $?" >> "$OUT/status.txt"
