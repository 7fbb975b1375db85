#!/bin/bash
# round 6 final tree, call B: kernel traces of the fused small-batch step (default HetroGIN and HetroGAT) -> the
# sb_busy records bench.py reports as kernel_ms_per_batch (placed in profiles/r06/ on this box too, so the bench line
# below reads this tree's), then the evidence half of tools/gpu_final.sh (the driver's bench command, rocprofv3
# summaries, aggregate PMC passes)
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r06_final_b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for spec in 'gin|' 'gat|--gat'; do
  IFS='|' read -r name extra <<< "$spec"
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$name" -o run -- \
    python3 tools/sb_prof.py --steps 200 $extra > "$OUT/trace_$name.log" 2>&1 || { tail -20 "$OUT/trace_$name.log"; exit 1; }
  python3 tools/sb_busy.py "$OUT/trace_$name" --steps 200 --label "$name" > "$OUT/sb_busy_$name.json" || exit 1
  cp "$OUT/sb_busy_$name.json" profiles/r06/sb_busy_$name.json
  head -8 "$OUT/sb_busy_$name.json"
done
SUITE=0 TAG=$TAG bash tools/gpu_final.sh
