#!/bin/bash
# round 6: fused HetroGAT step tests, GIN fused-step / GEMM-switch / bf16 / kernel suites (the pack_bf2 NaN branch),
# kernel-busy vs wall per batch (rocprofv3 kernel traces -> tools/sb_busy.py), bf16 GEMM A/B against the round-6 HEAD
# library (tools/ab/libhgin_head.so: before the pack_bf2 change)
set -o pipefail
TAG=${TAG:-r06e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch_gat.py \
  > $OUT/pytest_gat.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_gat.log | head -20; tail -3 $OUT/pytest_gat.log; exit 1; }
tail -2 $OUT/pytest_gat.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_smallbatch.py \
  tests/test_gpu_gemm_switch.py tests/test_gpu_bf16.py tests/test_gpu_kernels.py > $OUT/pytest_sb.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_sb.log | head -20; tail -3 $OUT/pytest_sb.log; exit 1; }
tail -2 $OUT/pytest_sb.log
for M in gin gat; do
  A=""; [ $M = gat ] && A="--gat"
  timeout -k 10 120 python -u tools/sb_prof.py --steps 200 $A > $OUT/sb_$M.out 2>&1 || { cat $OUT/sb_$M.out; exit 1; }
  cat $OUT/sb_$M.out
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$M -o run -- python3 tools/sb_prof.py --steps 200 $A \
    > $OUT/trace_$M.log 2>&1 || { tail -20 $OUT/trace_$M.log; exit 1; }
  python3 tools/sb_busy.py $OUT/trace_$M --steps 200 --label $M > $OUT/sb_busy_$M.json || exit 1
  head -8 $OUT/sb_busy_$M.json
done
for rep in 1 2; do
  for L in new head; do
    A=""; [ $L = head ] && A="--lib tools/ab/libhgin_head.so"
    timeout -k 10 120 python -u tools/gemm_ab.py --dtype bf16 --M 3000000 --reps 10 --only fwd256,fwd256acc,dx256,dw256pro,fwd512 $A >> $OUT/ab_pack.txt 2>&1 || exit 1
  done
done
grep '^{' $OUT/ab_pack.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d['lib'], {k:(v['ms'],v['GB_s']) for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
