#!/bin/bash
# dW split count after the one-launch slab sum: HGIN_TN_WGS 512 / 768 (default) / 1024, micro + cfg2 step.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-tn_wgs}
mkdir -p "$OUT"
for w in 768 512 1024 768; do
  HGIN_TN_WGS=$w timeout -k 10 200 python tools/slab_check.py > "$OUT/slab_$w.log" 2>&1 || { echo "FATAL slab $w"; exit 1; }
  HGIN_TN_WGS=$w timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/cfg2_$w.json" 2>/dev/null || { echo "FATAL bench $w"; exit 1; }
  echo "wgs=$w $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/cfg2_$w.json") ms/step"
  grep -h "tn_f32_cfg2\|mlpw_cfg2\|tn_bf16" "$OUT/slab_$w.log"
done
