#!/bin/bash
# A/B of the LDS-DMA gather aggregate (k_agg_lds, HGIN_AGG_LDS=1, ring depth D) against the register gather on cfg3:
# bench lines with the probe (aggregate TB/s from HIP events), then the variant tests.  Each step time-limited.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-agg_lds}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -20 "$OUT/$name.err"; exit $rc; }
}
run variants 600 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 300 --timeout-method thread -k "default or agg_lds"
run base 400 python bench.py --no-cpu-baseline --no-extras --steps 10
for D in ${DEPTHS:-8 12 16 24}; do
  HGIN_AGG_LDS=1 HGIN_AGG_LDS_D=$D run lds$D 400 python bench.py --no-cpu-baseline --no-extras --steps 10
done
for f in base $(for D in ${DEPTHS:-8 12 16 24}; do echo lds$D; done); do
  python3 -c "import json,sys; d=json.load(open('$OUT/$f.out')); r=d['roofline']; print('$f', d['ms_per_step'], r['achieved'], r['frac'], r['avg_launch_ms'])"
done
