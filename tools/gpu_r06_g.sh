#!/bin/bash
# round 6: the fused HetroGAT step with batched edge walks (gat_edges_x) — its tests, then ms per batch and a kernel trace
set -o pipefail
TAG=${TAG:-r06g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch_gat.py \
  > $OUT/pytest_gat.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_gat.log | head -20; tail -3 $OUT/pytest_gat.log; exit 1; }
tail -2 $OUT/pytest_gat.log
timeout -k 10 120 python -u tools/sb_prof.py --steps 200 --gat > $OUT/sb_gat.out 2>&1 || { cat $OUT/sb_gat.out; exit 1; }
cat $OUT/sb_gat.out
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_gat -o run -- python3 tools/sb_prof.py --steps 200 --gat \
  > $OUT/trace_gat.log 2>&1 || { tail -20 $OUT/trace_gat.log; exit 1; }
python3 tools/sb_busy.py $OUT/trace_gat --steps 200 --label gat > $OUT/sb_busy_gat.json || exit 1
head -16 $OUT/sb_busy_gat.json
