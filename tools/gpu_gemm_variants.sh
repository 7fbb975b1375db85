#!/bin/bash
# GEMM variant sweep on one GPU box: XCD-aware workgroup order on/off x split-M workgroup target.
# Each configuration is its own process (the switches are read once per process).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/gemm_variants
mkdir -p "$OUT"
for xcd in 1 0; do
  for wgs in 1024 768; do
    echo "=== HGIN_XCD=$xcd HGIN_TN_WGS=$wgs" >> "$OUT/fp32.txt"
    HGIN_XCD=$xcd HGIN_TN_WGS=$wgs timeout -k 10 200 python tools/gemm_bench.py --quick >> "$OUT/fp32.txt" 2>&1 || exit $?
    echo "=== HGIN_XCD=$xcd HGIN_TN_WGS=$wgs" >> "$OUT/bf16.txt"
    HGIN_XCD=$xcd HGIN_TN_WGS=$wgs timeout -k 10 200 python tools/gemm_bench_bf16.py --quick >> "$OUT/bf16.txt" 2>&1 || exit $?
  done
done
