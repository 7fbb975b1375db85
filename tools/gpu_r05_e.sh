#!/bin/bash
# Round 5 (e): the one-pass GAT attention forward — GAT tests, the relation profile and the extras line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gat.py tests/test_boundary.py -m "gpu or not gpu" -q --timeout 240 --timeout-method thread > $OUT/tests.out 2>&1 || { echo FAIL tests; tail -40 $OUT/tests.out; exit 1; }
tail -2 $OUT/tests.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_gat -o run -- python3 tools/extras_probe.py --only gat > $OUT/prof_gat.log 2>&1 || { echo FAIL prof_gat; tail -20 $OUT/prof_gat.log; exit 1; }
grep '"gat"' $OUT/prof_gat.log | tail -1 | cut -c1-900
f=$(find $OUT/prof_gat -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -c1-150
