#!/bin/bash
# Bench lines of the non-headline configs at HEAD: cfg2bf (cfg2 sizes, bf16) and cfg3 (100M edges, fp32).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-other_cfgs}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --config cfg2bf --no-cpu-baseline > "$OUT/bench_cfg2bf.json" 2> "$OUT/cfg2bf.err" || { echo "FATAL cfg2bf $?"; tail -5 "$OUT/cfg2bf.err"; exit 1; }
timeout -k 10 600 python bench.py --config cfg3 --no-cpu-baseline > "$OUT/bench_cfg3.json" 2> "$OUT/cfg3.err" || { echo "FATAL cfg3 $?"; tail -5 "$OUT/cfg3.err"; exit 1; }
for c in cfg2bf cfg3; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline']['frac'])" "$OUT/bench_$c.json"; done
