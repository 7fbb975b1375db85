#!/bin/bash
# Round 5 (c): GAT wave kernels (single-round-trip forward, parallel column sums) and the k_wsd_f32 split — tests,
# the GAT relation profile, per-launch A/B of the readout dW.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gat.py tests/test_gpu_kernels.py tests/test_gpu_gemm_switch.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/tests.out 2>&1 || { echo FAIL tests; tail -30 $OUT/tests.out; exit 1; }
tail -2 $OUT/tests.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_gat -o run -- python3 tools/extras_probe.py --only gat > $OUT/prof_gat.log 2>&1 || { echo FAIL prof_gat; tail -20 $OUT/prof_gat.log; exit 1; }
grep '"gat"' $OUT/prof_gat.log | tail -1 | cut -c1-900
timeout -k 10 300 python tools/gemm_ab.py --only dwro,dw256pro > $OUT/ab.out 2>&1 || { echo FAIL ab; tail -20 $OUT/ab.out; exit 1; }
cat $OUT/ab.out
