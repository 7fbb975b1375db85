#!/bin/bash
# round 6: n_parts A/B of the fused step (weight-gradient row chunks) at hidden 8 / 128 and for HetroGAT
set -u
OUT=gpurun_out/${TAG:-r06n}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch_gat.py \
  > "$OUT/pytest_gat.log" 2>&1 || { grep -E "^E |FAILED" "$OUT/pytest_gat.log" | head -20; tail -3 "$OUT/pytest_gat.log"; exit 1; }
tail -1 "$OUT/pytest_gat.log"
for spec in 'gin|{}|' 'h128|{"node_embedding_size": 128}|' 'gat|{}|--gat'; do
  IFS='|' read -r name model extra <<< "$spec"
  for np in 512 256 128 64 32; do
    timeout -k 10 120 python3 tools/sb_prof.py --steps 200 --model "$model" $extra --n-parts $np >> "$OUT/ab.log" 2>&1 || { tail -5 "$OUT/ab.log"; exit 1; }
  done
done
grep '^{' "$OUT/ab.log"
