#!/bin/bash
# round 6: PMC HBM traffic of the cfg5 bf16 GEMM kernels (k_ws_bf16 forward / dX, k_wsd_bf16 dW) — FETCH_SIZE and
# WRITE_SIZE in separate passes over the cfg5 bench command
set -u
OUT=gpurun_out/${TAG:-r06p}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_ws_bf16|k_wsd_bf16" --output-format csv \
      -d "$OUT/pmc_$C" -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras --steps 2 --warmup 1 \
      > "$OUT/pmc_$C.out" 2> "$OUT/pmc_$C.err" || { echo "FATAL pmc_$C"; tail -5 "$OUT/pmc_$C.err"; exit 1; }
done
echo done > "$OUT/status.txt"
