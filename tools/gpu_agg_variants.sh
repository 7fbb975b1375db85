#!/bin/bash
# Aggregate variant sweep: quads per lane (HGIN_AGG_NQ) x dtype, one process per configuration.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/agg_variants
mkdir -p "$OUT"
for nq in 0 2 4; do
  for dt in "" "--bf16"; do
    HGIN_AGG_NQ=$nq timeout -k 10 300 python tools/agg_bench.py $dt >> "$OUT/agg.txt" 2>&1 || exit $?
  done
done
