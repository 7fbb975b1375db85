#!/bin/bash
# round 6: the fused HetroGAT small-batch step (tests/test_gpu_smallbatch_gat.py), the GIN fused-step suite with the
# dead-relation Adam skip, the bf16 GEMM switch tests (k_ws_bf16 at 64 columns per wave), then kernel-busy vs wall per
# batch of the fused step (rocprofv3 kernel trace -> tools/sb_busy.py) for config.json's HetroGIN and HetroGAT
set -o pipefail
TAG=${TAG:-r06d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch_gat.py \
  > $OUT/pytest_gat.log 2>&1 || { tail -40 $OUT/pytest_gat.log; exit 1; }
tail -3 $OUT/pytest_gat.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_smallbatch.py \
  tests/test_gpu_gemm_switch.py > $OUT/pytest_sb.log 2>&1 || { tail -40 $OUT/pytest_sb.log; exit 1; }
tail -3 $OUT/pytest_sb.log
for M in gin gat; do
  A=""; [ $M = gat ] && A="--gat"
  timeout -k 10 120 python -u tools/sb_prof.py --steps 200 $A > $OUT/sb_$M.out 2>&1 || { cat $OUT/sb_$M.out; exit 1; }
  cat $OUT/sb_$M.out
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$M -o run -- python3 tools/sb_prof.py --steps 200 $A \
    > $OUT/trace_$M.log 2>&1 || { tail -20 $OUT/trace_$M.log; exit 1; }
  python3 tools/sb_busy.py $OUT/trace_$M --steps 200 --label $M > $OUT/sb_busy_$M.json || exit 1
  head -8 $OUT/sb_busy_$M.json
done
timeout -k 10 120 python -u tools/gemm_ab.py --dtype bf16 --M 3000000 --reps 10 --only fwd256,fwd256acc,dx256,dw256pro > $OUT/ab_default.txt 2>&1 || exit 1
tail -1 $OUT/ab_default.txt
