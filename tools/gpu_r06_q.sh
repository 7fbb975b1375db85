#!/bin/bash
# round 6: PMC HBM traffic of the cfg3 fp32 weight-stationary GEMMs (k_wss_f32 incl. the two-pass first-layer forward,
# k_wsp_f32 dW) — FETCH_SIZE and WRITE_SIZE in separate passes over the cfg3 bench command
set -u
OUT=gpurun_out/${TAG:-r06q}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_wss_f32|k_wsp_f32|k_ws_f32|k_wsd_f32|k_gemm_nt" --output-format csv \
      -d "$OUT/pmc_$C" -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --no-probe --no-extras --steps 2 --warmup 1 \
      > "$OUT/pmc_$C.out" 2> "$OUT/pmc_$C.err" || { echo "FATAL pmc_$C"; tail -5 "$OUT/pmc_$C.err"; exit 1; }
done
python3 tools/pmc_kernels.py "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" 3
