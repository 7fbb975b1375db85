#!/bin/bash
# round 6: kernel breakdown of the fused step's slower configs (hidden 128, MLP_BN) — rocprofv3 kernel traces
set -u
OUT=gpurun_out/${TAG:-r06l}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for spec in 'h128:{"node_embedding_size": 128}' 'bn:{"mlp_bn": true}'; do
  name=${spec%%:*}; model=${spec#*:}
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$name" -o run -- \
    python3 tools/sb_prof.py --steps 200 --model "$model" > "$OUT/trace_$name.log" 2>&1 || { tail -20 "$OUT/trace_$name.log"; exit 1; }
  grep ms_per_batch "$OUT/trace_$name.log"
  python3 tools/sb_busy.py "$OUT/trace_$name" --steps 200 --label "$name" > "$OUT/sb_busy_$name.json" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/sb_busy_$name.json')); print('$name', d['kernel_ms_per_batch'], d['wall_ms_per_batch']); [print('  ', k, v) for k, v in d['kernels_us'].items()]"
done
