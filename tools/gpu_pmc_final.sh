#!/bin/bash
# PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) over the cfg3 bench for the aggregate family and
# the fp32 weight-stationary GEMMs, at the final tree.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_agg|k_ws_f32" --output-format csv \
      -d "$OUT/pmc_$C" -o run -- python3 bench.py --no-cpu-baseline --no-probe --no-extras --steps 2 --warmup 1 \
      > "$OUT/pmc_$C.out" 2> "$OUT/pmc_$C.err"
  rc=$?; echo "pmc_$C $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL pmc_$C $rc"; tail -5 "$OUT/pmc_$C.err"; exit $rc; }
done
echo done >> "$OUT/status.txt"
