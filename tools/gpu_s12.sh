#!/bin/bash
# Round-3 s12: fp32 NT tile with the B image double-buffered (HGIN_NT_BDB=1): bitwise switch test, A/B timing on the
# cfg3 forward shapes.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s12}
mkdir -p "$OUT"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -6 "$OUT/$name.out"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step sw 600 python -u -m pytest tests/test_gpu_gemm_switch.py -x -q --timeout 400 --timeout-method thread -k "nt_m16 or default"
step ab_default 240 python tools/h2_bench.py
step ab_m16 240 env HGIN_NT_M16=1 python tools/h2_bench.py
echo done >> "$OUT/status.txt"
