#!/bin/bash
# round 6: fused small-batch step — 8-row forward blocks for wide layers, deeper operand batches where a weight comes
# through the caches: the fused-step suites, then kernel traces of the default / hidden 128 / MLP_BN / GAT steps
set -u
OUT=gpurun_out/${TAG:-r06m}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_smallbatch.py \
  tests/test_gpu_smallbatch_gat.py > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED" "$OUT/pytest.log" | head -20; tail -3 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for spec in 'gin|{}|' 'h128|{"node_embedding_size": 128}|' 'bn|{"mlp_bn": true}|' 'gat|{}|--gat'; do
  IFS='|' read -r name model extra <<< "$spec"
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$name" -o run -- \
    python3 tools/sb_prof.py --steps 200 --model "$model" $extra > "$OUT/trace_$name.log" 2>&1 || { tail -20 "$OUT/trace_$name.log"; exit 1; }
  timeout -k 10 120 python3 tools/sb_prof.py --steps 200 --model "$model" $extra > "$OUT/ev_$name.log" 2>&1 || exit 1
  grep ms_per_batch "$OUT/ev_$name.log"
  python3 tools/sb_busy.py "$OUT/trace_$name" --steps 200 --label "$name" > "$OUT/sb_busy_$name.json" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/sb_busy_$name.json')); print('$name', d['kernel_ms_per_batch'], d['wall_ms_per_batch']); [print('  ', k, v) for k, v in d['kernels_us'].items()]"
done
