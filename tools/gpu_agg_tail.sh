#!/bin/bash
# Aggregate neighbour-walk variants: batched tail on/off, rows in flight U = 8 / 16, fp32 / bf16; then the
# aggregate parity tests and cfg2 bench lines.  One process per setting (switches are read once).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-agg_tail}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -q -x -k aggregate --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo FAIL tests; tail $OUT/tests.txt; exit 1; }
for u in 8 16; do for dt in "" "--bf16"; do
  HGIN_AGG_U=$u timeout -k 10 300 python tools/agg_bench.py $dt >> $OUT/agg_u$u.txt 2>&1 || exit 1
done; done
for u in 8 16; do
  HGIN_AGG_U=$u timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_u$u.json 2>>$OUT/bench.err || exit 1
done
